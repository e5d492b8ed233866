"""The full-size reconstruction case shared by tests/golden/make_golden_fullsize.py (reference side)
and tests/test_fullsize_gpu.py (this package on cuda:0): SigLIP2-L at 512^2 and the f16d32
stage-0 Generator at 256^2 with tools/reconstruct/reconstruct.py's settings."""
import zlib

import torch

VFM_DIRNAME = "siglip2-large-patch16-512"
SIGLIP_L_CFG = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                    image_size=512, patch_size=16, num_channels=3, layer_norm_eps=1e-6)
REF_YAML = "vfm_vae_f16d32_siglip2_stage_0_strong_alignment.yaml"
# reference tools/reconstruct/reconstruct.py:106-113 (label_dim: 0 here, unconditional either way)
RECON_OVERRIDES = dict(img_resolution=256, conditional=False, label_type="cls2text", use_kl_loss=False,
                       use_vf_loss=False, num_fp16_res=0)
# the training backward (tests/golden/make_golden_fullsize_bwd.py): the stage-0 YAML's generator with its
# KL / VF losses on, fp32 decoder on the reference side (the CPU reference has no reduced-precision path)
TRAIN_OVERRIDES = dict(img_resolution=256, conditional=False, label_type="cls2text", num_fp16_res=0)
TRAIN_GROUPS = ("synthesis", "mapping", "ldm_adapter")      # what the G phase updates (VFM tower frozen)
R_SEED = 77
VF_W, KL_W = 3.0, 1e-3        # loss = sum(gen_img R) + sum_i sum(ms_i R_i) + VF_W vf + KL_W kl (terms of similar size)
HIDDEN_NAMES = ("h0", "h12", "hlast")      # patch_from_layers [0, 12, -1]
ROW_STRIDE = 16
IMG_SEED = 2024
EPS_SEED = 123


def image():
    """The 256^2 input in [0, 1] (CPU generator: the same values on every machine)."""
    return torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(IMG_SEED))


def psnr(a, b, peak=2.0):
    """PSNR of images in [-1, 1] (peak-to-peak 2)."""
    mse = float((a.double() - b.double()).square().mean())
    return float("inf") if mse == 0 else 10.0 * torch.log10(torch.tensor(peak * peak / mse)).item()


def loss_weights(img_shape, ms_shapes):
    """R (gen_img) and R_i (multiscale images) of the backward golden's loss: standard normal from a
    seeded CPU generator, so both sides draw the same values."""
    g = torch.Generator().manual_seed(R_SEED)
    R = torch.randn(tuple(img_shape), generator=g)
    return R, [torch.randn(tuple(s), generator=g) for s in ms_shapes]


P_SEED = 9001
# gradients stored whole (or every ROWSTEP-th output row) by the backward golden, next to every parameter's
# norm, sum and projection: one 1x1 weight per decoder block (the ConvNeXt MLP's second pointwise conv,
# every 32nd output row; block 5's whole), a square 1x1 of the latent stem, and the adapter's projections
FULL_GRADS = tuple((f"synthesis.blocks.{i}.conv0.pwconv2.weight", 32) for i in range(6)) + (
    ("synthesis.blocks.5.conv0.pwconv2.weight", 1),
    ("synthesis.z_convs.2.1.0.weight", 1),
    ("ldm_adapter.linear_proj.weight", 1),
    ("ldm_adapter.post_quant.blocks.0.proj.weight", 1),
    ("ldm_adapter.patch_quants.0.0.blocks.0.proj.weight", 1),
    ("ldm_adapter.patch_quants.0.0.blocks.0.attn.proj.weight", 1),
    ("ldm_adapter.final_quant.blocks.0.attn.proj.weight", 1),
)


NPROJ = 8                   # projections per parameter


def grad_probe(name, shape):
    """The NPROJ probes P_k of the projections <g, P_k> stored per parameter: standard normal, drawn in
    fp32 from a CPU generator seeded by the parameter's name (both sides draw the same values) and used
    in fp64 -> [NPROJ, *shape]. A gradient that is transposed, permuted or written to the wrong bucket
    keeps its norm and sum but moves each projection by ~N(0, |error|^2): the RMS over NPROJ of them
    estimates |error| (one projection alone lands below a quarter of |error| one time in five)."""
    g = torch.Generator().manual_seed(P_SEED ^ zlib.crc32(name.encode()))
    return torch.randn((NPROJ,) + tuple(shape), generator=g).double()


def projections(name, grad):
    """<g, P_k> for k < NPROJ (fp64)."""
    gd = grad.detach().double().cpu()
    return grad_probe(name, gd.shape).reshape(NPROJ, -1) @ gd.reshape(-1)


def grad_errors(name, grad, ref_norm, ref_proj, floor):
    """(norm error, projection error) of one parameter gradient against its golden values, both
    relative to max(|g_ref|, floor): |g| - |g_ref|, and the RMS over the NPROJ projections of
    <g - g_ref, P_k> (~ |g - g_ref| for any error; ~1.4 |g_ref| for a transposed gradient)."""
    gd = grad.detach().double().cpu()
    scale = max(float(ref_norm), floor, 1e-30)
    e_norm = abs(float(gd.norm()) - float(ref_norm)) / scale
    d = projections(name, gd) - torch.as_tensor(ref_proj, dtype=torch.float64)
    e_proj = float(d.square().mean().sqrt()) / scale
    return e_norm, e_proj


def full_grad_error(grad, ref, rowstep):
    """|g[::rowstep] - ref| / |ref| for a stored (row-subsampled) gradient."""
    gd = grad.detach().double().cpu()[::rowstep]
    ref = torch.as_tensor(ref).double()
    assert tuple(gd.shape) == tuple(ref.shape), (tuple(gd.shape), tuple(ref.shape))
    return float((gd - ref).norm() / max(float(ref.norm()), 1e-30))
