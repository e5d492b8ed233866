"""The DINOv2-L case shared by tests/golden/make_golden_dinov2.py (reference side) and tests/test_dinov2_gpu.py
(this package on cuda:0): BASELINE config 3's encoder (configs/vfm_vae_f16d32_dinov2_l_stage_0_dynres.yaml:
facebook/dinov2-large, scale_factor 0.875, patch_from_layers [0, 12, -1]) on the 256 / 384 / 512 stream and one
equivariance-prior downscale."""
import torch

VFM_DIRNAME = "dinov2-large"
# HF Dinov2Config of facebook/dinov2-large (the architecture; weights from tests/det_init.py)
DINOV2_L_CFG = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, mlp_ratio=4, patch_size=14,
                    image_size=518, num_channels=3, layer_norm_eps=1e-6, layerscale_value=1.0,
                    hidden_act="gelu", use_swiglu_ffn=False)
SCALE_FACTOR = 0.875
LAYERS = (0, 12, -1)
HIDDEN_NAMES = ("h0", "h12", "hlast")
ROW_STRIDE = 16
CASES = (dict(name="r256", res=256, eq_scale=1.0, prior=False, seed=31),
         dict(name="r384", res=384, eq_scale=1.0, prior=False, seed=32),
         dict(name="r512", res=512, eq_scale=1.0, prior=False, seed=33),
         dict(name="r256eq", res=256, eq_scale=0.5, prior=True, seed=34))


def image(res, seed):
    """A [1, 3, res, res] input in [0, 1] from a seeded CPU generator (the same values on every machine)."""
    return torch.rand(1, 3, res, res, generator=torch.Generator().manual_seed(seed))
