"""Graph replay vs eager at the full C1 size after a decoder weight update (the xfail case of
tests/test_configs_gpu.py::test_graph_replay_after_weight_update_c1), with every decoder module's
output recorded on both sides: forward hooks clone outputs eagerly in the eager runs and inside the
capture in the graphed run (the clones are graph nodes, refilled at every replay)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), os.path.join(ROOT, "tests"), ROOT]
os.environ["VFM_EXPERIMENTAL_GRAPHS"] = "1"
import torch  # noqa: E402

import test_configs_gpu as tc  # noqa: E402

if os.environ.get("GC1_NORM") == "mm":
    # channel norm through a GEMM instead of torch's reduction kernel (no global-reduce semaphores)
    from networks.utils import gigagan_utils

    def _norm_mm(self, x):
        B_, C_, H_, W_ = x.shape
        ones = torch.ones(1, 1, C_, device=x.device, dtype=x.dtype)
        ss = torch.matmul(ones, (x * x).reshape(B_, C_, H_ * W_))
        return x / ss.sqrt().clamp_min(1e-12).reshape(B_, 1, H_, W_) * self.scale * self.gamma

    gigagan_utils.ChannelRMSNorm.forward = _norm_mm

B = int(os.environ.get("GC1_B", "4"))
c, step = tc._build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = False
forced = (1.0, 0, False)
G.equivariance_transform.forced = forced
G.equivariance_transform.outcomes = lambda: [forced]
img, labels = tc._images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd

mode = ["graph"]
rec = {"graph": {}, "eager": {}}
order = []


def hook(name):
    def f(mod, inp, out):
        t = out[0] if isinstance(out, (tuple, list)) else out
        if isinstance(t, torch.Tensor) and t.is_cuda:
            rec[mode[0]][name] = t.detach().clone()
            if name not in order:
                order.append(name)
    return f


def pre(name):
    def f(mod, inp):
        t = inp[0] if inp else None
        if isinstance(t, torch.Tensor) and t.is_cuda:
            rec[mode[0]][name + ":in"] = t.detach().clone()
            if name + ":in" not in order:
                order.append(name + ":in")
        g = getattr(mod, "gamma", None)
        if isinstance(g, torch.Tensor):
            rec[mode[0]][name + ":gamma"] = g.detach().clone()
            if name + ":gamma" not in order:
                order.append(name + ":gamma")
    return f


for n, m in G.named_modules():
    if n and not n.startswith("vfm_encoder"):
        if n.endswith(".norm") or n.endswith("ff.0"):
            m.register_forward_pre_hook(pre(n))
        m.register_forward_hook(hook(n))


def ptrs():
    return {n: (p.data_ptr(), p.untyped_storage().data_ptr()) for n, p in G.named_parameters()}


def ptr_diff(tag, a, b):
    moved = [n for n in a if a[n] != b.get(n)]
    print(f"  params moved {tag}: {len(moved)} {moved[:6]}", flush=True)


SYNC = os.environ.get("GC1_SYNC", "0") == "1"


def rep():
    mode[0] = "graph"
    if SYNC:
        torch.cuda.synchronize()
    with torch.no_grad():
        torch.manual_seed(7)
        return gr(img, labels).gen_img.float().clone()


def eag():
    mode[0] = "eager"
    with torch.no_grad():
        torch.manual_seed(7)
        return G(img, labels).gen_img.float().clone()


def d(a, b):
    return float((a - b).abs().max())


def bisect(tag):
    torch.cuda.synchronize()
    bad = 0
    for n in order:
        a, b = rec["graph"].get(n), rec["eager"].get(n)
        if a is None or b is None or a.shape != b.shape:
            continue
        diff = d(a.float(), b.float())
        if diff != 0:
            print(f"  {tag} DIFF {n}: {diff:.3e} (|eager| max {float(b.float().abs().max()):.3e}) {tuple(b.shape)} {b.dtype}",
                  flush=True)
            bad += 1
            if bad >= 20:
                break
    print(f"  {tag}: modules {len(order)} mismatching (first 20 shown) {bad}", flush=True)


p0 = ptrs()
r0 = rep()
p1 = ptrs()
ptr_diff("by capture", p0, p1)
e0 = eag()
print("disabled", gr.disabled, "graphs", len(gr.graphs), flush=True)
print("before update: replay vs eager", d(r0, e0), "| gen max", float(e0.abs().max()), flush=True)
bisect("before")
with torch.no_grad():
    for p in G.synthesis.parameters():
        p.add_(1e-3 * torch.randn_like(p))
ptr_diff("by update", p1, ptrs())
o1 = rep()
e2 = eag()
ptr_diff("by eager after update", p1, ptrs())
bisect("o1")
e3 = eag()
o2 = rep()
bisect("o2")
print("after update: o1 vs e2", d(o1, e2), "| o2 vs e2", d(o2, e2), "| e3 vs e2", d(e3, e2),
      "| o1 vs r0", d(o1, r0), "| e2 vs e0", d(e2, e0), flush=True)
