"""The full-size reconstruction case shared by tests/golden/make_golden_fullsize.py (reference side)
and tests/test_fullsize_gpu.py (this package on cuda:0): SigLIP2-L at 512^2 and the f16d32
stage-0 Generator at 256^2 with tools/reconstruct/reconstruct.py's settings."""
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
