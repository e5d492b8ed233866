"""Loader for the gfx950 kernel library (`libvfmvae_hip.so`) behind `include/vfmvae.h`.

Replaces the reference's JIT plugin builder `torch_utils/custom_ops.py:59-155`
(`get_plugin`: torch.utils.cpp_extension.load of .cpp/.cu sources into an
md5-keyed cache). Here the kernels are prebuilt in-tree by `csrc/Makefile`
(`__graft_entry__.build()`), the binding is ctypes over the plain C ABI, and a
missing or unloadable library is a hard error: there is no silent fallback for
GPU tensors.
"""
import ctypes
import os
import threading

import torch

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libvfmvae_hip.so")
# A/B builds of the same library (tools_dev experiments): VFM_HIP_LIB names another in-tree build in lib/
if os.environ.get("VFM_HIP_LIB"):
    _LIB_PATH = os.path.join(os.path.dirname(_LIB_PATH), os.path.basename(os.environ["VFM_HIP_LIB"]))
# TORCH_LIBRARY(vfmvae) registration of the reference's plugin ops (csrc/torch_ops.cpp)
_TORCH_LIB_PATH = os.path.join(os.path.dirname(_LIB_PATH), "libvfmvae_torch.so")
_torch_ops = None
_lock = threading.RLock()          # get_torch_ops holds it while it calls get_native
_lib = None

c_int, c_ll, c_float, c_vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p
c_llp = ctypes.POINTER(ctypes.c_longlong)
c_fp = ctypes.POINTER(ctypes.c_float)

# name -> argtypes (restype is always int). Keep in sync with include/vfmvae.h.
SIGNATURES = {
    "vfm_upfirdn2d": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_llp, c_int, c_int, c_llp,
                      c_int, c_int, c_ll, c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_vp],
    "vfm_bias_act": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_int, c_int, c_float, c_float, c_float,
                     c_ll, c_int, c_vp],
    "vfm_filtered_lrelu": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_llp,
                           c_int, c_int, c_llp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_int, c_vp],
    "vfm_filtered_lrelu_act": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_llp, c_int, c_int, c_int,
                               c_int, c_int, c_float, c_float, c_float, c_vp],
    "vfm_dwconv2d_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_dwconv2d_bwd_weight_tiles": [c_int, c_int, c_int, c_int, c_int, c_int],
    "vfm_dwconv2d_bwd_weight": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_group_norm_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_float, c_vp],
    "vfm_group_norm_fwd_stats": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_float, c_vp],
    "vfm_group_norm_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                           c_int, c_int, c_int, c_vp],
    "vfm_scale_bias_gelu_fwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_scale_bias_gelu_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_layer_scale_residual_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_layer_scale_residual_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                     c_vp],
    "vfm_shuffle_blur_fwd": [c_vp, c_vp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_shuffle_blur_bwd": [c_vp, c_vp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_codebook_argmax": [c_vp, c_ll, c_vp, c_int, c_int, c_int, c_vp, c_vp],
    "vfm_residual_layer_norm": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_vp],
    "vfm_layer_norm_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp],
    "vfm_layer_norm_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp],
    "vfm_pw_gemm_gelu": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                         c_vp],
    "vfm_pw_gemm_gelu_tiles": [c_int],
    "vfm_convnext_mlp_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                             c_int, c_vp],
    "vfm_lpips_head_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_lpips_head_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_lpips_head_fwd_nhwc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_lpips_head_bwd_nhwc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_gemm8": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int, c_ll,
                  c_ll, c_ll, c_ll, c_float, c_float, c_int, c_int, c_vp, c_int, c_int, c_vp],
    "vfm_gemm8_pieces": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll,
                         c_int, c_ll, c_ll, c_ll, c_ll, c_ll, c_float, c_float, c_int, c_int, c_vp, c_int, c_int,
                         c_vp],
    "vfm_gemm8_workspace_floats": [c_int, c_int, c_int, c_int, c_int, c_int, c_int],
    "vfm_gemm8_set_schedule": [c_int],
    "vfm_gemm8_gelu": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                       c_ll, c_ll, c_ll, c_ll, c_ll, c_vp],
    "vfm_gemm8_gelu_parts": [c_int],
    "vfm_gemm8_set_stamps": [c_vp],
    "vfm_channel_rms_norm_rows": [c_int, c_int, c_int],
    "vfm_channel_rms_norm_fwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp],
    "vfm_channel_rms_norm_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp],
    "vfm_style_demod_fwd": [c_vp, c_ll, c_vp, c_vp, c_vp, c_float, c_float, c_float, c_int, c_int, c_int, c_int,
                            c_vp, c_vp, c_vp, c_vp],
    "vfm_style_demod_bwd_workspace_floats": [c_int, c_int, c_int, c_int],
    "vfm_style_demod_bwd": [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_float, c_int, c_int,
                            c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "vfm_dwconv2d_fwd_ex": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_vp],
    "vfm_dwconv2d_fwd_mfma_ex": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_vp],
    "vfm_dwconv2d_fwd_mfma_nz": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_vp],
    "vfm_dwconv2d_fwd_mfma_units": [c_int, c_int, c_int, c_int, c_int, c_int],
    "vfm_dwconv2d_fwd_mfma_gs": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_vp],
    "vfm_dwconv2d_wgrad_reduce": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp],
    "vfm_specnorm_workspace_floats": [c_int, c_int],
    "vfm_specnorm_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_float, c_vp],
    "vfm_specnorm_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp],
    "vfm_im2col1d_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_col2im1d_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_im2col1d_cbl_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_col2im1d_cbl_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_colsum2_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp],
    "vfm_shift2d": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_im2col_nhwc_f32": [c_vp, c_vp, c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_col2im_nhwc_f32": [c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_int, c_vp],
    "vfm_rowdot_f32": [c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_vp],
    "vfm_coldot_splits": [c_int, c_int],
    "vfm_coldot_f32": [c_vp, c_ll, c_vp, c_vp, c_int, c_int, c_int, c_vp],
    "vfm_bnl_workspace_floats": [c_int, c_int, c_int, c_int],
    "vfm_bnl_lrelu_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_float,
                          c_vp],
    "vfm_bnl_lrelu_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                          c_float, c_vp],
    "vfm_dwconv2d_fwd_mfma": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_posterior_fwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_posterior_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp],
    "vfm_dwconv2d_bwd_weight_mfma_tiles": [c_int, c_int, c_int, c_int, c_int, c_int],
    "vfm_dwconv2d_bwd_weight_mfma": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_bnl1d_lrelu_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_float, c_vp],
    "vfm_bnl1d_lrelu_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_vp],
    "vfm_torgb_fwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_torgb_bwd_splits": [c_int, c_int, c_int],
    "vfm_torgb_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_split_f32": [c_vp, c_vp, c_int, c_int, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_vp],
    "vfm_gemm_workspace_floats": [c_int, c_int, c_int, c_int, c_int],
    "vfm_gemm": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int,
                 c_ll, c_ll, c_ll, c_ll, c_float, c_float, c_int, c_int, c_int, c_int, c_vp],
    "vfm_attention_fwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_llp, c_llp, c_llp, c_llp, c_float,
                          c_vp],
    "vfm_conv3x3_dgrad_small_f32": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "vfm_maxpool2x2_nhwc_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_maxpool2x2_bwd_nhwc_f32": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_conv3x3_nhwc_f32": [c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_vp],
    "vfm_attention_f32_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_llp, c_llp, c_llp,
                              c_llp, c_float, c_int, c_vp],
    "vfm_gemm9_set_mode": [c_int],
    "vfm_gemm9_gelu": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_ll,
                       c_ll, c_ll, c_ll, c_ll, c_vp],
    "vfm_gemm9_gelu_parts": [c_int],
    "vfm_gemm9_ex": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int, c_ll, c_ll, c_ll,
                     c_float, c_vp, c_int, c_int, c_vp],
    "vfm_gemm9_workspace_floats": [c_int, c_int, c_int, c_int, c_int, c_int],
    "vfm_gemm9_pieces": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_int, c_ll, c_ll,
                         c_ll, c_ll, c_ll, c_float, c_int, c_vp, c_int, c_int, c_vp],
    "vfm_gemm9": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int, c_ll, c_ll,
                  c_ll, c_ll, c_float, c_float, c_int, c_int, c_vp],
    "vfm_sgemm": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int, c_ll, c_ll, c_ll, c_ll,
                  c_float, c_float, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp],
    "vfm_sgemm_workspace_floats": [c_int, c_int, c_int, c_int, c_int],
    "vfm_timer_mode": [c_int],
    "vfm_im2col2d_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_vp],
    "vfm_col2im2d_f32": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_vp],
    "vfm_timer_null_launch": [c_vp],
    "vfm_adam_chunk_elems": [],
    "vfm_style_group_bytes": [c_int],
    "vfm_specnorm_group_bytes": [c_int],
    "vfm_group_norm_fwd_pc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_float, c_vp],
    "vfm_scale_bias_gelu_fwd_pc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_scale_bias_gelu_bwd_pc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "vfm_layer_scale_residual_bwd_pc": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                        c_int, c_vp],
    "vfm_dwconv2d_fwd_res": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_vp],
    "vfm_specnorm_group_pack": [c_int, c_int, c_vp, c_vp, c_vp, c_vp],
    "vfm_specnorm_group_launch": [c_int, c_vp, c_int, c_ll, c_vp],
    "vfm_style_group_pack": [c_int, c_int, c_vp, c_vp, c_vp, c_vp],
    "vfm_style_group_launch": [c_int, c_vp, c_int, c_ll, c_vp],
    "vfm_adam_ema_step": [c_vp, c_int, c_vp, c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                          ctypes.c_double, ctypes.c_double, ctypes.c_double, c_float, c_vp],
    "vfm_adam_ema_step_raw": [c_vp, c_int, c_vp, c_int, c_vp, c_float, c_int, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              c_float, c_vp],
    "vfm_timer_arm_first": [c_vp, c_vp],
    "vfm_gemm_fold": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll,
                      c_ll, c_float, c_float, c_int, c_int, c_vp],
    "vfm_timer_arm": [c_vp, c_vp],
    "vfm_event_create": [ctypes.POINTER(c_vp)],
    "vfm_event_destroy": [c_vp],
    "vfm_event_elapsed": [c_vp, c_vp, c_fp],
    "vfm_attention_f32_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                              c_int, c_llp, c_llp, c_llp, c_llp, c_llp, c_llp, c_llp, c_llp, c_float, c_int, c_vp],
}

DTYPE_CODES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3}
VFM_NO_KERNEL = -1
VFM_F32, VFM_BF16, VFM_F32X3 = 0, 2, 4

# Products of fp32 operands on the MFMA paths (GEMMs, the VGG conv, fp32 attention):
#   "f32x6" (default): three exact bf16 pieces per operand, the six piece products of order
#           >= 2^-16, fp32 accumulation -- fp32-equivalent (dropped terms <= ~2^-23 relative),
#           the precision of the reference's fp32 legs (TF32 off, training_loop.py:504-505);
#   "f32x3" (opt-in, VFM_F32_PRODUCTS=f32x3): hi / lo pieces, three products, ~2^-15.5 relative.
F32_PRODUCTS = os.environ.get("VFM_F32_PRODUCTS", "f32x6")
if F32_PRODUCTS not in ("f32x6", "f32x3"):
    raise ValueError(f"VFM_F32_PRODUCTS must be f32x6 or f32x3, not {F32_PRODUCTS!r}")


def f32_precision():
    """(ABI precision code, piece count, region tag) of the fp32 product mode."""
    return (VFM_F32, 3, "f32x6") if F32_PRODUCTS == "f32x6" else (VFM_F32X3, 2, "f32x3")


class _NoCtx:
    """The ctx a FastFunction's forward gets when it runs outside autograd: saving is a no-op and no
    input needs a gradient (`needs_input_grad` is a tuple of False, one per forward argument, so
    indexing and slicing behave as on autograd's ctx); attributes may be set (and are dropped with the
    object)."""
    __slots__ = ("needs_input_grad", "__dict__")

    def __init__(self, nargs):
        self.needs_input_grad = (False,) * nargs

    def save_for_backward(self, *tensors):
        pass

    def mark_non_differentiable(self, *tensors):
        pass

    def set_materialize_grads(self, value):
        pass


class FastFunction(torch.autograd.Function):
    """autograd.Function whose apply() with grad mode off calls forward directly: what apply would
    do there too (no graph node, outputs without grad_fn), minus its ~8-10 us of host work per call,
    which the no-grad generator forward of the D phase pays ~10^3 times per step while the GPU waits
    for the host (tools_dev/gapprof.py)."""

    @classmethod
    def apply(cls, *args, **kwargs):
        if torch.is_grad_enabled():
            return super().apply(*args, **kwargs)
        return cls.forward(_NoCtx(len(args) + len(kwargs)), *args, **kwargs)


class NativeError(RuntimeError):
    pass


def library_path():
    return _LIB_PATH


def get_native():
    """Load (once) and return the ctypes handle of the kernel library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_LIB_PATH):
                raise NativeError(
                    f"HIP kernel library not found at {_LIB_PATH}; run `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(or `make -C vfm-vae_amd/csrc`)")
            lib = ctypes.CDLL(_LIB_PATH)
            for name, argtypes in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = argtypes
                fn.restype = c_int
            lib.vfm_version.restype = ctypes.c_char_p
            lib.vfm_bnl_workspace_floats.restype = c_ll
            lib.vfm_gemm9_workspace_floats.restype = c_ll
            lib.vfm_sgemm_workspace_floats.restype = c_ll
            lib.vfm_style_group_bytes.restype = c_ll
            lib.vfm_specnorm_group_bytes.restype = c_ll
            lib.vfm_specnorm_group_pack.restype = c_ll
            lib.vfm_style_group_pack.restype = c_ll
            lib.vfm_channel_rms_norm_rows.restype = c_ll
            lib.vfm_specnorm_workspace_floats.restype = c_ll
            lib.vfm_dwconv2d_fwd_mfma_units.restype = c_ll
            _lib = lib
    return _lib


def get_torch_ops():
    """Load (once) the TORCH_LIBRARY(vfmvae) library and return `torch.ops.vfmvae`: upfirdn2d,
    bias_act, filtered_lrelu, filtered_lrelu_act_ with the reference plugins' schemas
    (upfirdn2d.cpp:102-105, bias_act.cpp:94-97, filtered_lrelu.cpp:295-299 of the reference).
    A missing library is a hard error."""
    global _torch_ops
    if _torch_ops is not None:
        return _torch_ops
    get_native()                          # outside the lock: it takes the lock itself
    with _lock:
        if _torch_ops is None:
            if not os.path.exists(_TORCH_LIB_PATH):
                raise NativeError(f"torch op library not found at {_TORCH_LIB_PATH}; run the build "
                                  "(`make -C vfm-vae_amd/csrc`)")
            torch.ops.load_library(_TORCH_LIB_PATH)
            _torch_ops = torch.ops.vfmvae
    return _torch_ops


def get_plugin(module_name=None, sources=None, headers=None, source_dir=None, **_build_kwargs):
    """Reference-compatible entry point (`custom_ops.get_plugin`): returns the
    prebuilt native library regardless of the source list."""
    return get_native()


def dtype_code(t: torch.Tensor) -> int:
    try:
        return DTYPE_CODES[t.dtype]
    except KeyError:
        raise NativeError(f"unsupported dtype {t.dtype}")


def strides(t: torch.Tensor):
    arr = (ctypes.c_longlong * t.ndim)(*t.stride())
    return arr


def strides_of(values):
    """ctypes long long array of arbitrary element strides."""
    return (ctypes.c_longlong * len(values))(*values)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """hipStream_t of the current stream (the raw handle, without building a Stream object:
    this runs once per kernel launch)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        else:
            idx = device.index if isinstance(device, torch.device) else int(device)
            if idx is None:
                idx = torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def check(rc: int, name: str, allow_no_kernel: bool = False) -> int:
    if rc == 0 or (allow_no_kernel and rc == VFM_NO_KERNEL):
        return rc
    raise NativeError(f"{name} failed with code {rc}")
