"""Network / loss parity against golden vectors produced by the reference itself
(tests/golden/make_golden_networks.py). CPU, fp32: this package's modules,
with the same name-keyed weights (tests/det_init.py), must reproduce the
reference Generator / ProjectedDiscriminator / LPIPS outputs and the gradients
of one full D + G `accumulate_gradients` step.

Tolerances: outputs 1e-4 of max magnitude (fp32, different but equivalent op
decompositions: batched GEMM instead of grouped conv for the modulated 1x1,
fused qkv, explicit patch-embed GEMM); gradient norms 1e-3 relative.
"""
import json
import os

import numpy as np
import pytest
import torch

import golden_io
import net_cases
from det_init import det_init, canonical

G_FILE = "networks_golden.npz"


def _arr(k):
    return golden_io.load(G_FILE)[0][k]


def _meta():
    return golden_io.load(G_FILE)[1]


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


@pytest.fixture(scope="module")
def vfm_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("vfm") / net_cases.VFM_DIRNAME
    d.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(d / "config.json", "w"))
    return str(d)


def _check_grads(prefix, module, names_key=None, norm_tol=1e-3, full_tol=2e-3, sum_tol=1e-3, scalar_tol=None):
    """Every parameter gradient of `module` (any device) against the reference's norms,
    sums and (where stored) full tensors. Returns the worst relative norm error."""
    names = [canonical(n) for n in _meta()[f"{prefix}/grad_names"]]
    sums, norms = _arr(f"{prefix}/grad_sum"), _arr(f"{prefix}/grad_norm")
    params = {canonical(n): p for n, p in module.named_parameters()}
    got = {n: p for n, p in params.items() if p.grad is not None}
    assert set(got) == set(names), (set(got) ^ set(names))
    worst = 0.0
    floor = 1e-4 * float(np.max(norms))        # grads that are ~0 in exact math (bias before a norm layer)
    for n, s, nm in zip(names, sums, norms):
        g = got[n].grad.detach().double().cpu()
        scale = max(nm, floor, 1e-12)
        err = abs(float(g.norm()) - nm) / scale
        worst = max(worst, err)
        ntol, stol = norm_tol, sum_tol
        if scalar_tol is not None and g.numel() == 1:
            ntol = stol = scalar_tol
        assert err < ntol, (n, float(g.norm()), nm)
        assert abs(float(g.sum()) - s) <= stol * scale * max(1.0, g.numel() ** 0.5), (n, float(g.sum()), s)
        arrays = golden_io.load(G_FILE)[0]
        key = next((k for k in (f"{prefix}/grad/{n}", f"{prefix}/grad/{n.replace('vision_model.', 'vision_model.vision_model.', 1)}") if k in arrays), None)
        if key is not None:
            ref = np.asarray(arrays[key], np.float64)
            assert float(np.abs(g.numpy() - ref).max()) <= (max(full_tol, ntol) if g.numel() == 1 else full_tol) * max(float(np.abs(ref).max()), floor), n
    return worst


@pytest.fixture(scope="module")
def generator(vfm_dir):
    from networks.generator import Generator
    torch.manual_seed(0)
    G = Generator(label_dim=0, **net_cases.g_kwargs(vfm_dir)).train()
    det_init(G)
    return G


def test_generator_state_dict_keys_match_reference(generator):
    assert sorted(canonical(k) for k in generator.state_dict().keys()) == sorted(canonical(k) for k in _meta()["G_state_keys"])
    assert generator.num_ws == _meta()["G_num_ws"]


def test_generator_forward_backward_matches_reference(generator):
    G = generator
    G.zero_grad(set_to_none=True)
    G.requires_grad_(False)
    for m in (G.synthesis, G.mapping, G.ldm_adapter):
        m.requires_grad_(True)
    img = torch.from_numpy(_arr("G/img"))
    torch.manual_seed(123)
    out = G(img, ['x'] * 2, validation=True)
    assert _rel(out.gen_img.detach(), _arr("G/gen_img")) < 1e-4
    for i, m in enumerate(out.gen_multiscale_imgs):
        assert _rel(m.detach(), _arr(f"G/ms{i}")) < 1e-4, i
    assert _rel(out.vf_loss.detach(), _arr("G/vf_loss")) < 1e-5
    assert _rel(out.kl_loss.detach(), _arr("G/kl_loss")) < 1e-5
    R = torch.from_numpy(_arr("G/R"))
    Rs = [torch.from_numpy(_arr(f"G/R{i}")) for i in range(len(out.gen_multiscale_imgs))]
    loss = (out.gen_img * R).sum() + sum((m * r).sum() for m, r in zip(out.gen_multiscale_imgs, Rs)) \
        + 3.0 * out.vf_loss + 1e3 * out.kl_loss
    loss.backward()
    _check_grads("G", G)


def test_discriminator_matches_reference():
    from networks.discriminator import ProjectedDiscriminator
    D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train()
    det_init(D)
    assert sorted(D.state_dict().keys()) == _meta()["D_state_keys"]
    x = torch.from_numpy(_arr("D/x")).requires_grad_(True)
    out = D(x, None)
    assert _rel(out.stylegan_t_logits.detach(), _arr("D/logits")) < 1e-4
    for s, scale in enumerate(out.patchgan_logits):
        assert _rel(scale[-1].detach(), _arr(f"D/patch{s}")) < 1e-4
        sums = _meta()[f"D/patch{s}_feat_sums"]
        for t, ref in zip(scale, sums):
            assert abs(float(t.detach().double().sum()) - ref) <= 1e-4 * max(1.0, abs(ref)) + 1e-3 * t.numel() ** 0.5
    R = torch.from_numpy(_arr("D/R"))
    dl = (out.stylegan_t_logits * R).sum() + sum(s[-1].square().mean() for s in out.patchgan_logits)
    dl.backward()
    assert _rel(x.grad, _arr("D/dx")) < 1e-3
    _check_grads("D", D)


def test_lpips_matches_reference():
    from training.lpips import LPIPS
    L = LPIPS().eval()
    det_init(L)
    a = torch.from_numpy(_arr("L/a"))
    b = torch.from_numpy(_arr("L/b")).requires_grad_(True)
    v = L(a, b)
    assert _rel(v.detach(), _arr("L/val")) < 1e-5
    v.sum().backward()
    assert _rel(b.grad, _arr("L/db")) < 1e-4


def test_total_loss_step_matches_reference(vfm_dir):
    from networks.generator import Generator
    from networks.discriminator import ProjectedDiscriminator
    from training.loss import TotalLoss
    torch.manual_seed(5)
    G2 = Generator(label_dim=0, **net_cases.g_kwargs(vfm_dir)).train().requires_grad_(False)
    D2 = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train().requires_grad_(False)
    det_init(G2)
    det_init(D2)
    loss = TotalLoss(device=torch.device('cpu'), G=G2, D=D2, **net_cases.loss_kwargs(vfm_dir))
    det_init(loss.perceptual_module)
    real = torch.from_numpy(_arr("T/real"))
    D2.requires_grad_(True)
    D2.dino.requires_grad_(False)
    torch.manual_seed(321)
    loss.accumulate_gradients(phase='D', real_img=real, real_c=['x'] * 2, cur_nimg=0)
    D2.requires_grad_(False)
    _check_grads("T/D", D2, norm_tol=2e-3, full_tol=1e-2)
    for name, layer in G2.named_modules():
        layer.requires_grad_(any(t in name for t in G2.trainable_layers))
    torch.manual_seed(654)
    loss.accumulate_gradients(phase='G', real_img=real, real_c=['x'] * 2, cur_nimg=0)
    ref = _meta()["T/prev_loss_dict"]
    for k, v in ref.items():
        assert abs(loss.prev_loss_dict[k] - v) <= 1e-4 * max(1.0, abs(v)), k
    _check_grads("T/G", G2, norm_tol=2e-3, full_tol=1e-2)
    assert loss._off_done    # PatchGAN on -> reconstruction losses switched off after the step (reference semantics)
