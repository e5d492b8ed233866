"""Locate the first module whose output differs between the eager no-grad G forward and its
HIP-graph replay (training/graphed_forward.py). Forward hooks clone every module output:
eagerly in the reference run, inside the capture in the graphed run (the clones are graph
nodes, filled at replay)."""
import json
import os
import random
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import net_cases  # noqa: E402
from networks.generator import Generator  # noqa: E402
from training.graphed_forward import GraphedNoGradForward  # noqa: E402

rec = {}
order = []


def hook(name):
    def f(mod, inp, out):
        t = out[0] if isinstance(out, (tuple, list)) else out
        if isinstance(t, torch.Tensor) and t.is_cuda:
            rec[name] = t.detach().clone()
            if name not in order:
                order.append(name)
    return f


def main():
    d = os.path.join(tempfile.mkdtemp(), net_cases.VFM_DIRNAME)
    os.makedirs(d)
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(os.path.join(d, "config.json"), "w"))
    torch.manual_seed(0)
    G = Generator(label_dim=0, **net_cases.g_kwargs(d, use_equivariance_regularization=False)).train() \
        .requires_grad_(False).cuda()
    for n, m in G.named_modules():
        if n:
            m.register_forward_hook(hook(n))
    img = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(5)).cuda()
    x0 = G.mapping.x_avg.clone()
    random.seed(1)
    torch.manual_seed(1)
    with torch.no_grad():
        ref = G(img, ['x', 'x']).gen_img.clone()
    eager = dict(rec)
    G.mapping.x_avg.copy_(x0)
    runner = GraphedNoGradForward(G)
    random.seed(1)
    torch.manual_seed(1)
    with torch.no_grad():
        rec.clear()
        runner(img, ['x', 'x'])       # captures (hooks record graph-pool clones), then replays
    print("disabled:", runner.disabled, "graphs:", len(runner.graphs))
    torch.cuda.synchronize()
    ent = next(iter(runner.graphs.values()))
    print("noise buffers:", [tuple(b.shape) for b in getattr(ent, 'bufs', [])])
    torch.manual_seed(1)
    for b in getattr(ent, 'bufs', []):
        e = torch.randn(b.shape)
        print("eps buffer vs first draw after seed: max diff", float((b.cpu() - e).abs().max()),
              "buffer absmax", float(b.abs().max()))
    print("graph gen_img vs eager:", float((ent.out.gen_img - ref).abs().max()))
    bad = 0
    for n in order:
        if n in eager and n in rec and eager[n].shape == rec[n].shape:
            diff = float((eager[n].float() - rec[n].float()).abs().max())
            if diff != 0:
                print(f"DIFF {n}: {diff:.3e} shape {tuple(eager[n].shape)} {eager[n].dtype}")
                bad += 1
                if bad > 25:
                    break
    print("modules compared:", len(order), "mismatching:", bad)


if __name__ == "__main__":
    main()
