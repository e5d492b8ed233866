/*
 * vfmvae.h — C ABI of the MI355X (gfx950) VFM-VAE hot-path kernels.
 *
 * This is the drop-in boundary that replaces the reference's pybind11 plugins
 * (`torch_utils/custom_ops.py:59-155` building `upfirdn2d_plugin`,
 * `bias_act_plugin`, `filtered_lrelu_plugin`) and the torch/cuDNN calls of the
 * decoder layers that actually run in the shipped configs
 * (`networks/utils/convnext_utils.py:36-257`).
 *
 * Conventions (all entry points):
 *   - Plain device pointers, element counts and element strides; no torch types.
 *   - Outputs are allocated by the caller (the Python host layer allocates them
 *     from PyTorch's caching allocator, like `torch::empty` in the reference's
 *     host code, e.g. `upfirdn2d.cpp:38`).
 *   - Kernels are enqueued asynchronously on `stream` (a hipStream_t; NULL is the
 *     legacy default stream). No host synchronisation, no allocation: every entry
 *     point is capturable into a hipGraph.
 *   - Return value: VFM_OK (0) on success, VFM_ERR_ARGS (-2) for an invalid
 *     argument, VFM_NO_KERNEL (-1) when no specialisation exists (only
 *     `vfm_filtered_lrelu`, mirroring `filtered_lrelu.cpp:51-56`), or a positive
 *     hipError_t from the launch.
 *   - dtype codes: VFM_F32, VFM_F16, VFM_BF16, VFM_F64. Arithmetic is fp32
 *     (fp64 for VFM_F64); filters are always fp32.
 */
#ifndef VFMVAE_H
#define VFMVAE_H

#ifdef __cplusplus
extern "C" {
#endif

enum {
    VFM_F32 = 0,
    VFM_F16 = 1,
    VFM_BF16 = 2,
    VFM_F64 = 3,
    /* Precision code of the fp32 MFMA paths only (GEMM / conv / fp32 attention): fp32 operands as
     * the opt-in 3-term bf16 split (hi.hi + hi.lo + lo.hi, ~2^-15.5 relative per product). VFM_F32
     * on those paths is the fp32-equivalent 6-term split (three exact bf16 pieces per operand, the
     * six products of order >= 2^-16; dropped terms <= ~2^-23 relative, fp32 accumulation). */
    VFM_F32X3 = 4,
};

enum {
    VFM_OK = 0,
    VFM_NO_KERNEL = -1,
    VFM_ERR_ARGS = -2,
};

/* Library identification: returns a static string "vfmvae-hip <version> gfx950". */
const char* vfm_version(void);

/*
 * Kernel timing (measurement only; no reference counterpart). While (start, stop) is armed on the
 * calling thread, every kernel the library launches is dispatched with hipExtLaunchKernelGGL and the
 * two events bound to the dispatch itself: start = the first launch's start, stop = the end of each
 * launch. hipEventElapsedTime(start, stop) is then the kernels' own duration (no host launch gaps).
 * vfm_timer_arm(NULL, NULL) disarms; every call returns the number of launches made under the
 * previous arming (0: the events were not recorded). Events come from vfm_event_create.
 */
int vfm_timer_arm(void* start, void* stop);
/* Start-event binding of the armed timer: 1 (default) = the end of an empty probe kernel launched right before
 * each timed kernel (the interval excludes the previous kernel's tail the timed one waits behind); 0 = the
 * timed kernel's own dispatch (hipExtLaunchKernelGGL start event). Returns the previous mode. */
int vfm_timer_mode(int mode);
/* One empty kernel launch through the library's launch path (timed when armed): calibration of the fixed
 * interval every timed launch carries (dispatch gap + an empty one-wave kernel). */
int vfm_timer_null_launch(void* stream);
/* vfm_timer_arm timing only the FIRST launch of the call (a GEMM's main kernel, not its split-K combine pass). */
int vfm_timer_arm_first(void* start, void* stop);
int vfm_event_create(void** ev);
int vfm_event_destroy(void* ev);
int vfm_event_elapsed(void* start, void* stop, float* ms);

/*
 * upfirdn2d: upsample (zero insertion) -> pad/crop -> 2-D FIR -> downsample -> gain.
 * Replaces `upfirdn2d(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1,
 * flip, gain)` of `torch_utils/ops/upfirdn2d.cpp:16` (kernels `upfirdn2d.cu:29-200`).
 *   x: [N, C, inH, inW] with element strides xs[4] (N, C, H, W order); any layout.
 *   y: [N, C, outH, outW] with element strides ys[4]; the caller computes
 *      outW = (inW*upx + padx0 + padx1 - fw + downx) / downx (same for H).
 *   f: fp32 filter [fh, fw] with element strides (fsh, fsw).
 *   flip: 0 = convolution, 1 = correlation (reference `flip_filter`).
 */
int vfm_upfirdn2d(const void* x, void* y, const float* f, int dtype,
                  int N, int C, int inH, int inW, const long long* xs,
                  int outH, int outW, const long long* ys,
                  int fh, int fw, long long fsh, long long fsw,
                  int upx, int upy, int downx, int downy, int padx0, int pady0,
                  int flip, float gain, void* stream);

/*
 * bias_act: y = clamp(act(x + b[(i / stepB) % sizeB]) * gain) and its 1st/2nd
 * order gradients. Replaces `bias_act(x, b, xref, yref, dy, grad, dim, act,
 * alpha, gain, clamp)` of `torch_utils/ops/bias_act.cpp:32` (kernel
 * `bias_act.cu:23-147`). All tensors are dense with the same element order;
 * NULL = absent (the reference passes empty tensors). act codes follow
 * `bias_act.py:21-31` (1 linear, 2 relu, 3 lrelu, 4 tanh, 5 sigmoid, 6 elu,
 * 7 selu, 8 softplus, 9 swish); clamp < 0 disables clamping.
 */
int vfm_bias_act(const void* x, const void* b, const void* xref, const void* yref,
                 const void* dy, void* y, int dtype, long long numel,
                 int grad, int act, float alpha, float gain, float clamp,
                 long long stepB, int sizeB, void* stream);

/*
 * filtered_lrelu: bias -> upsample FIR (gain up^2) -> gain -> leaky ReLU ->
 * clamp -> downsample FIR, fused. Replaces `filtered_lrelu(x, fu, fd, b, si, up,
 * down, px0, px1, py0, py1, sx, sy, gain, slope, clamp, flip_filters,
 * writeSigns)` of `torch_utils/ops/filtered_lrelu.cpp:16`.
 *   x: [N, C, xh, xw] (strides xs), y: [N, C, yh, yw] (strides ys), both dtype.
 *   fu: fp32 [fuh, fuw] contiguous, fd: fp32 [fdh, fdw] contiguous (separable
 *       filters are passed as their 2-D outer product).
 *   b: [C] dtype (may be NULL = zero bias).
 *   s: uint8 sign tensor [N, C, sh, sw_bytes] contiguous; written when
 *      sign_mode == 1, read (at offset sx, sy) when sign_mode == 2, unused (NULL)
 *      when sign_mode == 0. 2 bits per element: bit0 = negative, bit1 = clamped.
 *   clamp: use +inf for "no clamp".
 * Returns VFM_NO_KERNEL when (up, down) is outside {1,2,4} or the tile would not
 * fit in LDS; the host layer then takes the generic path
 * (upfirdn2d -> vfm_filtered_lrelu_act -> upfirdn2d), as `filtered_lrelu.py:223-229`.
 */
int vfm_filtered_lrelu(const void* x, const float* fu, const float* fd, const void* b,
                       unsigned char* s, void* y, int dtype,
                       int N, int C, int xh, int xw, const long long* xs,
                       int yh, int yw, const long long* ys,
                       int fuh, int fuw, int fdh, int fdw,
                       int up, int down, int px0, int py0,
                       int sh, int sw_bytes, int sx, int sy, int sign_mode,
                       float gain, float slope, float clamp, int flip, void* stream);

/*
 * filtered_lrelu_act_: in-place gain -> leaky ReLU -> clamp on x [N, C, H, W]
 * (strides xs) with sign write (sign_mode 1) / read at offset (sx, sy)
 * (sign_mode 2). Replaces `filtered_lrelu_act_` of `filtered_lrelu.cpp:213`.
 * s: uint8 [N, C, sh, sw_bytes] contiguous.
 */
int vfm_filtered_lrelu_act(void* x, unsigned char* s, int dtype,
                           int N, int C, int H, int W, const long long* xs,
                           int sh, int sw_bytes, int sx, int sy, int sign_mode,
                           float gain, float slope, float clamp, void* stream);

/* Channel RMS norm of the decoder attention blocks (replaces F.normalize(x, dim=1) * scale * gamma of
 * reference networks/utils/gigagan_utils.py:31-39 ChannelRMSNorm): fp32 contiguous [B, C, P];
 * rinv [B, P] = 1 / max(||x||, 1e-12) saved for the backward (may be null in the forward). The
 * backward writes dx, and dgamma [C] through the workspace gpart [vfm_channel_rms_norm_rows, C]
 * (both null: no gamma gradient). */
long long vfm_channel_rms_norm_rows(int B, int C, int P);
int vfm_channel_rms_norm_fwd(const float* x, const float* gamma, float* y, float* rinv, int B, int C, int P,
                             float scale, void* stream);
int vfm_channel_rms_norm_bwd(const float* x, const float* gamma, const float* rinv, const float* dy, float* dx,
                             float* gpart, float* dgamma, int B, int C, int P, float scale, void* stream);

/* Style affine + demodulation coefficients of a ConvNeXt synthesis layer (replaces StyleSplit /
 * FullyConnectedLayer of reference networks/utils/shared.py and the demodulation of
 * networks/utils/convnext_utils.py:60-66): m = wg w A^T + bg ab [B, 3C], s = m1 m2 + m3 [B, C],
 * d = rsqrt(s^2 (W1^2)^T + eps) [B, O] (W1 null: no d). fp32; w rows ldw apart. The backward takes
 * dL/ds (ds_in) and dL/dd (dd) and writes any of dw [B, WD], dA [3C, WD], dab [3C], dW1 [O, C]
 * (null: skipped); ws is its workspace of vfm_style_demod_bwd_workspace_floats(B, C, WD, O) floats
 * (ds and the fixed-order partial sums of the column reductions; required). */
int vfm_style_demod_bwd_workspace_floats(int B, int C, int WD, int O);
int vfm_style_demod_fwd(const float* w, long long ldw, const float* A, const float* ab, const float* W1, float wg,
                        float bg, float eps, int B, int C, int WD, int O, float* m, float* s, float* d, void* stream);
int vfm_style_demod_bwd(const float* w, long long ldw, const float* A, const float* W1, const float* m,
                        const float* s, const float* d, const float* ds_in, const float* dd, float wg, float bg,
                        int B, int C, int WD, int O, float* ws, float* dW1, float* dA, float* dab, float* dw,
                        void* stream);
/* The style path of every ConvNeXt layer of a synthesis network in one launch per phase (forward launches 0, 1;
 * backward 2, 4, 3, 5, in that order; torch_utils/ops/style_group.py): vfm_style_group_pack writes launch `launch`'s
 * layer table and block offsets for n layers into host memory (vfm_style_group_bytes(n) bytes; per layer 16 pointer
 * slots w, A, ab, W1, m, s, d, ds_in, dd, ws, dW1, dA, dab, dw, ldw, lddw (dw's row stride), dims B, C, WD, O and
 * gains wg, bg, eps, as the single-layer calls above take them) and returns its total blocks; the caller uploads
 * the bytes and vfm_style_group_launch runs them. Same arithmetic per layer as the single-layer calls. */
long long vfm_style_group_bytes(int n);
long long vfm_style_group_pack(int launch, int n, const long long* ptrs, const int* dims, const float* gains,
                               void* host_out);
int vfm_style_group_launch(int launch, const void* dev_packed, int n, long long total_blocks, void* stream);

/* Spectral normalisation in training mode (torch.nn.utils.spectral_norm, one power iteration, dim 0: the
 * projected discriminator heads' SpectralConv1d, reference networks/discriminator.py): for fp32 W [O, I],
 * v <- normalize(W^T u), u <- normalize(W v) in place (copies to u_copy / v_copy when given), sigma [1] =
 * u . (W v), Wsn = W / sigma. The backward: dW = g / sigma - (sum g W) / sigma^2 u v^T. ws: workspace of
 * vfm_specnorm_workspace_floats floats. */
long long vfm_specnorm_workspace_floats(int O, int I);
int vfm_specnorm_fwd(const float* W, float* u, float* v, float* u_copy, float* v_copy, float* sigma, float* Wsn,
                     float* ws, int O, int I, float eps, void* stream);
int vfm_specnorm_bwd(const float* g, const float* W, const float* u, const float* v, const float* sigma, float* dW,
                     float* ws, int O, int I, void* stream);
/* Grouped spectral norm: every weight of the discriminator heads in one launch per phase (forward phases 0-2,
 * backward 3-4; torch_utils/ops/specnorm_group.py). vfm_specnorm_group_pack writes phase `phase`'s table for n
 * weights into host memory (vfm_specnorm_group_bytes(n) bytes; per weight 10 pointer slots W, u, v, u_copy, v_copy,
 * sigma, Wsn, ws, g, dW, dims O, I and eps) and returns its total blocks; the caller uploads the bytes and
 * vfm_specnorm_group_launch runs them. Same arithmetic per weight as vfm_specnorm_fwd / _bwd. */
long long vfm_specnorm_group_bytes(int n);
long long vfm_specnorm_group_pack(int phase, int n, const long long* ptrs, const int* dims, const float* eps,
                                  void* host_out);
int vfm_specnorm_group_launch(int phase, const void* dev_packed, int n, long long total_blocks, void* stream);

/* im2col of a 1-D conv with zero / circular padding and its adjoint, fp32 (the D heads' k = 9
 * SpectralConv1d, padding_mode='circular', reference networks/discriminator.py make_block):
 * cols [B, C k, Lo] (Lo = L + 2 p - k + 1; circular needs Lo == L) from x [B, C, L]; VFM_NO_KERNEL
 * for shapes not covered. */
int vfm_im2col1d_f32(const float* x, float* cols, int B, int C, int L, int k, int p, int circular, void* stream);
int vfm_col2im1d_f32(const float* dcols, float* dx, int B, int C, int L, int k, int p, int circular, void* stream);
/* the same gather / adjoint with the batch folded into the columns, cols [C k, B, Lo]: the head conv of the
   whole batch as one GEMM and its weight gradient as one GEMM with the batch in the reduction */
int vfm_im2col1d_cbl_f32(const float* x, float* cols, int B, int C, int L, int k, int p, int circular, void* stream);
int vfm_col2im1d_cbl_f32(const float* dcols, float* dx, int B, int C, int L, int k, int p, int circular,
                         void* stream);

/* Column sums of the per-sample [rows, cols] fp32 partials of the decoder backward kernels, two at a
 * time in one launch: out_a = scale_a * sum_r a (scale_a optional), out_b = sum_r b (either output may
 * be null); rows summed in order. */
int vfm_colsum2_f32(const float* a, const float* b, const float* scale_a, float* out_a, float* out_b, int rows,
                    int cols, void* stream);

/* DiffAugment random translation (replaces the padded gather of reference training/diffaug.py
 * rand_translation and its indexing backward): y[b, c, i, j] = x[b, c, i + sign tx[b], j + sign ty[b]]
 * inside the image, else 0; x, y contiguous NCHW (VFM_F32 / VFM_BF16); tx, ty int64 [B] on the device.
 * The backward is the same call with sign = -1. */
int vfm_shift2d(const void* x, void* y, const long long* tx, const long long* ty, int dtype, int B, int C, int H,
                int W, int sign, void* stream);

/* ---------------------------------------------------------------------------
 * Decoder ops (ConvNeXt synthesis layer, separable upsampler). The reference runs
 * these as stock torch modules; the entry points below replace the calls at
 *   networks/utils/convnext_utils.py:121-142  (ConvNeXtSynthesisLayer.forward:
 *       dwconv -> noise -> GroupNorm32 -> modulated pwconv1 -> GELU -> pwconv2 -> gamma -> residual)
 *   networks/utils/convnext_utils.py:234-257  (SeparableUpsampleWithFixedBlur.forward:
 *       GroupNorm -> depthwise 3x3 -> pointwise -> PixelShuffle -> replicate pad -> blur)
 *   networks/utils/shared.py:165-167          (GroupNorm32.forward, fp32 statistics)
 * All tensors are contiguous NCHW ([B, C, P] for the row ops); per-channel
 * vectors and filters are fp32; dtype codes as above (F32/F16/BF16).
 * ------------------------------------------------------------------------- */

/* Depthwise KxK conv (K in {1,3,5,7}), stride 1, zero padding `pad`, optional
 * fp32 bias [C] and additive plane noise [Ho, Wo]; w: fp32 [C, K, K].
 * y: [B, C, Ho, Wo], Ho = H + 2 pad - K + 1. The data gradient is this call
 * with dy, the flipped kernel and pad' = K - 1 - pad. */
int vfm_dwconv2d_fwd(const void* x, const float* w, const float* bias, const float* noise, void* y,
                     int dtype, int B, int C, int H, int W, int K, int pad, void* stream);

/* Number P of partial slots per channel the weight-gradient kernel writes. */
int vfm_dwconv2d_bwd_weight_tiles(int B, int C, int H, int W, int K, int pad);

/* Weight/bias gradient partials: partial[P, C, K*K + 1] (last slot = bias; P from
 * vfm_dwconv2d_bwd_weight_tiles). The caller sums over P in a fixed order (deterministic). */
int vfm_dwconv2d_bwd_weight(const void* x, const void* dy, float* partial, int dtype,
                            int B, int C, int H, int W, int K, int pad, void* stream);

/* y = ((x - mean) * rstd * w[c] + b[c]) * s[b, c], statistics over each of the
 * G groups of C/G channels x HW (fp32); w, b, s may be NULL. mean/rstd: [B*G]
 * fp32 outputs (saved for the backward). Input and output dtypes may differ. */
int vfm_group_norm_fwd(const void* x, const float* w, const float* b, const float* s, void* y,
                       float* mean, float* rstd, int dtype_in, int dtype_out,
                       int B, int C, int G, int HW, float eps, void* stream);
/* vfm_group_norm_fwd that also writes an fp32 y's exact bf16 pieces [3][B C HW] (16-B aligned, HW % 8 == 0) for
 * the f32x6 GEMM it feeds: the fp32 ConvNeXt layers' GN(d) * s, pwconv1's input (reference
 * networks/utils/convnext_utils.py:117-138). */
int vfm_group_norm_fwd_pc(const void* x, const float* w, const float* b, const float* s, void* y, void* y_pieces,
                          float* mean, float* rstd, int dtype_in, int dtype_out, int B, int C, int G, int HW,
                          float eps, void* stream);
/* vfm_group_norm_fwd (bf16 x) with each group's statistics merged, in double and a fixed order,
 * from the producer's per-wave partials stats [B C upc][4] (vfm_dwconv2d_fwd_mfma_gs; upc = units
 * per (sample, channel) plane) instead of a pass over x: x is read once. */
int vfm_group_norm_fwd_stats(const void* x, const float* w, const float* b, const float* s, void* y,
                             float* mean, float* rstd, const float* stats, int upc, int dtype_in, int dtype_out,
                             int B, int C, int G, int HW, float eps, void* stream);

/* GroupNorm backward: dx (dtype_x); dw_part/db_part [B, C] per-sample
 * contributions to d_weight / d_bias; ds [B, C] (when s != NULL). */
int vfm_group_norm_bwd(const void* x, const void* dy, const float* mean, const float* rstd,
                       const float* w, const float* b, const float* s, void* dx,
                       float* dw_part, float* db_part, float* ds,
                       int dtype_x, int dtype_dy, int B, int C, int G, int HW, void* stream);

/* g = gelu_erf(h * scale[b, o] + bias[o]) on h [B, O, P] (P % 8 == 0);
 * scale / bias may be NULL. */
int vfm_scale_bias_gelu_fwd(const void* h, const float* scale, const float* bias, void* g,
                            int dtype, int B, int O, int P, void* stream);

/* Backward: dh; d_scale_rows [B*O] = sum_p dz * h (NULL to skip), d_bias_rows [B*O] = sum_p dz. */
int vfm_scale_bias_gelu_bwd(const void* h, const void* dg, const float* scale, const float* bias,
                            void* dh, float* d_scale_rows, float* d_bias_rows,
                            int dtype, int B, int O, int P, void* stream);

/* out = x_in + gamma[c] * (y + bias[c]) on [B, C, P] (P % 8 == 0); out has x_in's dtype. */
int vfm_layer_scale_residual_fwd(const void* y, const float* bias, const float* gamma, const void* x_in,
                                 void* out, int dtype_y, int dtype_x, int B, int C, int P, void* stream);

/* Backward: dy = gamma * dout; d_gamma_rows [B*C] = sum_p (y + bias) dout; d_sum_rows [B*C] = sum_p dout. */
int vfm_layer_scale_residual_bwd(const void* y, const float* bias, const float* gamma, const void* dout,
                                 void* dy, float* d_gamma_rows, float* d_sum_rows,
                                 int dtype_y, int dtype_x, int B, int C, int P, void* stream);
/* The same three kernels writing, with an fp32 output, also its exact bf16 pieces (hi, mid, lo) as the planar
 * [3][numel] operand of the f32x6 GEMMs (`*_pieces`, 16-B aligned; bit-identical to vfm_split_f32's planar
 * split): the fp32 ConvNeXt layers' pwconv2 input g, pwconv1's output gradient dh and pwconv2's output gradient
 * dy (reference networks/utils/convnext_utils.py:135-142) enter their 1x1 products without a split pass. */
int vfm_scale_bias_gelu_fwd_pc(const void* h, const float* scale, const float* bias, void* g, void* g_pieces,
                               int dtype, int B, int O, int P, void* stream);
int vfm_scale_bias_gelu_bwd_pc(const void* h, const void* dg, const float* scale, const float* bias, void* dh,
                               void* dh_pieces, float* d_scale_rows, float* d_bias_rows, int dtype, int B, int O,
                               int P, void* stream);
int vfm_layer_scale_residual_bwd_pc(const void* y, const float* bias, const float* gamma, const void* dout, void* dy,
                                    void* dy_pieces, float* d_gamma_rows, float* d_sum_rows, int dtype_y,
                                    int dtype_x, int B, int C, int P, void* stream);

/* PixelShuffle(r) (r = 1: none) + replicate pad ((K-1)/2 before, K/2 after) + blur
 * with the separable normalised taps[K] (K <= 8; HOST pointer, read at launch):
 * x [B, C r^2, H, W] -> y [B, C, H r, W r]. */
int vfm_shuffle_blur_fwd(const void* x, void* y, const float* taps, int K, int dtype,
                         int B, int C, int H, int W, int r, void* stream);

/* Exact adjoint of vfm_shuffle_blur_fwd: dout [B, C, H r, W r] -> dx [B, C r^2, H, W]. */
int vfm_shuffle_blur_bwd(const void* dout, void* dx, const float* taps, int K, int dtype,
                         int B, int C, int H, int W, int r, void* stream);

/* ---------------------------------------------------------------------------
 * Frozen ViT towers (SigLIP2 encoder): fused residual add + LayerNorm, replacing the
 * torch `h + delta.float()` / `F.layer_norm(h).to(bf16)` pairs of the HF SiglipEncoderLayer
 * under bf16 autocast (networks/utils/vfms/siglip2_utils.py:114-137).
 *   h: fp32 [rows, D]; delta: [rows, D] (dtype_delta) or NULL; h_out: fp32 [rows, D]
 *   receives h + delta (NULL: not written; ignored when delta is NULL);
 *   y: [rows, D] (dtype_out) = LayerNorm(h + delta) * w + b (fp32 statistics, eps);
 *   w, b: fp32 [D] or NULL. D a multiple of 256, at most 2048 (else VFM_NO_KERNEL).
 * Forward only (the towers are frozen and run without autograd). */
int vfm_residual_layer_norm(const float* h, const void* delta, float* h_out, const float* w, const float* b,
                            void* y, int dtype_delta, int dtype_out, int rows, int D, float eps, void* stream);

/* LayerNorm with a backward, for a tower whose parameters are frozen but whose input needs a gradient
 * (the DINOv2 discriminator backbone in the G phase; reference HF Dinov2Layer norm1 / norm2, replaces
 * torch's layer_norm / layer_norm_backward there). x fp32 [rows, D], D a multiple of 128, at most 1024
 * (else VFM_NO_KERNEL); y [rows, D] (dtype_out); mean / rstd fp32 [rows] saved for the backward.
 * Backward: dx fp32 = rstd (g - mean(g) - xhat mean(g xhat)), g = dy w (dy in dtype_dy); no gradient for
 * w / b. Pointers 8-B aligned. */
int vfm_layer_norm_fwd(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                       int dtype_out, int rows, int D, float eps, void* stream);
int vfm_layer_norm_bwd(const float* x, const void* dy, const float* w, const float* mean, const float* rstd,
                       float* dx, int dtype_dy, int rows, int D, void* stream);

/* ---------------------------------------------------------------------------
 * Frozen ViT towers: fused multi-head self-attention forward (flash-style).
 * Replaces `F.scaled_dot_product_attention(q, k, v)` of HF SiglipAttention under bf16
 * autocast (reference networks/utils/vfms/siglip2_utils.py:121, SiglipVisionModel forward)
 * and of the DINOv2 / CLIP towers (configs 0, 3).
 *   q, k, v, o: bf16 [B, N, H, head_dim] views; sq/sk/sv/so = element strides
 *   {batch, token, head} (multiples of 8; unit stride along head_dim; 16-B aligned bases).
 *   o = softmax(q k^T * scale) v, fp32 softmax statistics, P rounded to bf16 for P.V.
 * head_dim 64 only (else VFM_NO_KERNEL). Forward only. */
int vfm_attention_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int N, int head_dim,
                      const long long* sq, const long long* sk, const long long* sv, const long long* so,
                      float scale, void* stream);

/* 3x3 / stride 1 / pad 1 convolution, NHWC fp32, implicit GEMM on bf16 MFMA with fp32-equivalent
 * products (precision VFM_F32: the 6-term split; VFM_F32X3: the opt-in 3-term one). Replaces the
 * MIOpen fp32 convolutions of the LPIPS VGG16 stack, reference training/lpips.py:126-163, forward
 * and data gradient. x [B, H, W, Cin] (Cin a power of two >= 4), w [Cout][9][Cin] (tap-major,
 * Cout % 64 == 0) given as its bf16 pieces w_pieces [np][Cout][ldw] (np = 3: hi = bf16(w),
 * mid = bf16(w - hi), lo = bf16(w - hi - mid); np = 2: hi, lo; rows zero-padded to ldw, a multiple
 * of 64 >= 9*Cin), out [B, H, W, Cout] = relu?(conv + bias), zeroed where mask [B, H, W, Cout] <= 0
 * when mask is given (bias / mask may be null). */
int vfm_conv3x3_nhwc_f32(const float* x, const void* w_pieces, int precision, int ldw, const float* bias,
                         const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int relu, void* stream);
/* Input gradient of a 3x3 / pad 1 conv with few input channels (the VGG16 image layer, C = 3), exact fp32
 * FMAs on the VALU (replaces torch.nn.grad.conv2d_input = MIOpen fp32 Winograd there):
 *   dx[b, c, y, x] = sum_{o, ky, kx} w[o, c, ky, kx] dz[b, y + 1 - ky, x + 1 - kx, o].
 * dz NHWC fp32 [B, H, W, K] (K % 4 == 0, K <= 128, 16-B aligned), w fp32 [K][C][3][3] (torch layout of
 * the forward weight), dx NCHW fp32 [B, C, H, W], C <= 4 (else VFM_NO_KERNEL). Deterministic. */
int vfm_conv3x3_dgrad_small_f32(const float* dz, const float* w, float* dx, int B, int H, int W, int C, int K,
                                void* stream);
/* 2x2 / stride-2 max pooling of the LPIPS VGG16 stack (torchvision vgg16().features nn.MaxPool2d(2, 2),
 * reference training/lpips.py:126-163) on NHWC fp32 [B, H, W, C] (C % 4 == 0, H and W even, 16-B
 * aligned; else VFM_NO_KERNEL): forward without indices (torch's rule: strictly greater or NaN replaces
 * the running max, rows then columns), and the backward fused with the tap gradient gt (NHWC, may be
 * NULL) and the ReLU derivative of the conv below: dx = (argmax ? g : 0 + gt) * (x > 0), the argmax
 * recomputed from the pool input x. Bit-identical to torch's max_pool2d_with_indices(_backward) + add
 * + mask chain. */
int vfm_maxpool2x2_nhwc_f32(const float* x, float* y, int B, int H, int W, int C, void* stream);
int vfm_maxpool2x2_bwd_nhwc_f32(const float* g, const float* x, const float* gt, float* dx, int B, int H, int W,
                                int C, void* stream);

/* fp32 attention with gradients (replaces F.scaled_dot_product_attention on the fp32 paths of the
 * generator: fusion-adapter AttnProjection, reference networks/utils/ldm_utils.py:55-93 (encode,
 * 64-dim heads; decode post_quant, 32-dim heads), the decoder SelfAttention with null key/value,
 * reference networks/utils/gigagan_utils.py:53-91, and the DINO discriminator tower).
 * q [B, Nq, H, d], k/v [B, Nk, H, d] fp32 views, d in {32, 64}, element strides {batch, token,
 * head}, unit stride on the head dim, strides multiples of 4, pointers 16-B aligned. Products run on
 * bf16 MFMA with fp32-equivalent products (precision VFM_F32: 6-term split; VFM_F32X3: opt-in 3-term),
 * fp32 accumulation and softmax.
 *   fwd: o (strides so) and lse [B, H, Nq] (log2 domain of the scaled scores);
 *   bwd: dq/dk/dv (own strides) from dout; delta [B, H, Nq] fp32 scratch. */
int vfm_attention_f32_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int H, int Nq,
                          int Nk, int head_dim, const long long* sq, const long long* sk, const long long* sv,
                          const long long* so, float scale, int precision, void* stream);
int vfm_attention_f32_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const void* lse, void* delta, void* dq, void* dk, void* dv, int B, int H, int Nq, int Nk,
                          int head_dim, const long long* sq, const long long* sk, const long long* sv,
                          const long long* so, const long long* sdo, const long long* sdq, const long long* sdk,
                          const long long* sdv, float scale, int precision, void* stream);

/* ---------------------------------------------------------------------------
 * Dense GEMM on the MFMA cores with a fused epilogue (replaces the hipBLASLt GEMMs behind
 * torch.addmm / torch.bmm for the frozen ViT projections, reference
 * networks/utils/vfms/siglip2_utils.py:121 (HF SiglipEncoderLayer q/k/v/o, fc1 + gelu_tanh,
 * fc2), the fusion adapter (ldm_utils.py:55-166), the decoder's 1x1 convolutions
 * (convnext_utils.py:36-142, gigagan_utils.py:53-185) and the discriminators' linears / convs):
 *   C[z] = epi(alpha * A[z] . B[z] + beta * C[z]), A: M x K, B: K x N, z < batch,
 *   epi = (+ bias[n] if bias_mode 1 | + bias[m] if bias_mode 2), then GELU (act 1 tanh,
 *   act 2 erf); fp32 accumulation.
 *   in_dtype VFM_BF16: bf16 operands; VFM_F32: fp32 operands, fp32-equivalent products (the 6-term
 *   bf16 split, see VFM_F32X3 above); VFM_F32X3: fp32 operands on the opt-in 3-term split.
 *   out_dtype VFM_BF16 / VFM_F32. Operand layouts: a_kcont = 1: A is [M][K] (row stride lda),
 *   0: A is [K][M]; b_kcont = 1: B is [N][K], 0: B is [K][N]; C is [M][N] (row stride ldc);
 *   sA/sB/sC = element batch strides (0 = shared operand). The contiguous extents, lda/ldb
 *   and sA/sB must be multiples of 8 (bf16) / 4 (fp32) elements (else VFM_NO_KERNEL).
 *   splits > 1: K split over workgroups; partial tiles go to `workspace` (fp32, at least
 *   vfm_gemm_workspace_floats(...) elements) and are summed in a fixed order by a second
 *   kernel that applies the epilogue. reduce_batch = 1: C (single matrix) = epi(sum over z)
 *   -- the weight gradient of a batched 1x1 convolution. */
int vfm_gemm_workspace_floats(int M, int N, int batch, int splits, int reduce_batch);
int vfm_gemm(const void* A, const void* B, void* C, const float* bias, float* workspace, int in_dtype,
             int out_dtype, int M, int N, int K, int batch, int a_kcont, long long lda, long long sA,
             int b_kcont, long long ldb, long long sB, long long ldc, long long sC, float alpha, float beta,
             int bias_mode, int act, int splits, int reduce_batch, void* stream);
/* Batch-folded form of vfm_gemm for a shared A (sA = 0, either layout): C[z] = epi(alpha A B[z] + beta C[z]),
 * z < batch, B[z] MN-contiguous [K][P] (row stride ldb, batch stride sB), C[z] [M][P] (row stride ldc,
 * batch stride sC), P = 2^lgp >= 8 columns per sample, run as ONE product over N = batch * P columns
 * (column n -> sample n >> lgp): per-sample planes narrower than a 128-wide tile -- the 1x1
 * convolutions of the 8 x 8 decoder block (reference networks/utils/convnext_utils.py:36-142,
 * gigagan_utils.py:53-185 at 8 x 8) -- fill whole tiles. bias_mode 2: per row; 1: per column of the
 * P-wide plane. No split-K, no workspace. */
int vfm_gemm_fold(const void* A, const void* B, void* C, const float* bias, int in_dtype, int out_dtype, int M,
                  int lgp, int K, int batch, int a_kcont, long long lda, long long ldb, long long sB, long long ldc,
                  long long sC, float alpha, float beta, int bias_mode, int act, void* stream);

/* im2col of a 2-D convolution (kernel kh x kw, stride (sy, sx), zero padding (py, px), dilation 1) over an NCHW
 * fp32 x [B, C, H, W] into cols [B, C kh kw, Ho Wo] (Ho = (H + 2 py - kh) / sy + 1, likewise Wo), and its adjoint
 * (col2im: x = the sum of the cols entries that read each element, a gather: deterministic, overwrites x).
 * With vfm_sgemm they form the convolution of reference torch_utils/ops/conv2d_resample.py:46-141
 * (conv2d_gradfix.conv2d / conv_transpose2d, conv2d_gradfix.py:37-58) and generator.py:46-103's grouped
 * modulated_conv2d (torch_utils/ops/conv2d_hip.py). */
int vfm_im2col2d_f32(const float* x, float* cols, int B, int C, int H, int W, int kh, int kw, int sy, int sx, int py,
                     int px, int Ho, int Wo, void* stream);
int vfm_col2im2d_f32(const float* cols, float* x, int B, int C, int H, int W, int kh, int kw, int sy, int sx, int py,
                     int px, int Ho, int Wo, void* stream);

/* One launch for a phase's optimizer step (csrc/adam.hip): Adam (torch.optim.Adam's fused arithmetic, ORIGINAL
 * weight decay) over every tensor of the device table `tensors` (ntensors 64-B records {p, g, m, v, ema or null, n,
 * vec, fp32 step counter or null: advanced by 1 in the launch}) through the chunk list `chunks` (nchunks int pairs
 * (tensor, chunk) of vfm_adam_chunk_elems() elements),
 * and for records with an EMA copy the G_ema lerp ema <- ema + ema_w (p - ema) on the stepped p. bc1 =
 * 1 - beta1^step, bc2_sqrt = sqrt(1 - beta2^step). Replaces the reference's opt.step() + G_ema lerp (reference
 * training/training_loop.py:722-742; host side training_loop.fast_adam_step / torch_utils/ops/adam_hip.py). */
int vfm_adam_chunk_elems(void);
int vfm_adam_ema_step(const void* tensors, int ntensors, const void* chunks, int nchunks, double lr, double beta1,
                      double beta2, double weight_decay, double eps, double bc1, double bc2_sqrt, float ema_w,
                      void* stream);
/* The same step with the gradients read through `grads` (device array of ntensors float pointers replacing the
 * records' g; null: the records' g) and, when clean != 0, used as nan_to_num(g * gscale) (nan 0, +inf 1e5, -inf
 * -1e5): the gradient scaling and cleanup of FlatGradSync.finish() (reference training/training_loop.py:281-289,
 * sync_grads' gain and nan_to_num over the flat gradient) applied as the raw per-step gradient tensors are read. */
int vfm_adam_ema_step_raw(const void* tensors, int ntensors, const void* chunks, int nchunks, const void* grads,
                          float gscale, int clean, double lr, double beta1, double beta2, double weight_decay,
                          double eps, double bc1, double bc2_sqrt, float ema_w, void* stream);

/* Exact-fp32 form of the vfm_gemm contract on the fp32-input MFMA (csrc/sgemm.hip, v_mfma_f32_32x32x2_f32: one
 * fmaf-chain product per multiply-add, no operand split): C[z] = epi(alpha A[z] B[z] + beta C[z]), fp32 A / B / C,
 * bias (1 per column, 2 per row) then act (1 gelu tanh, 2 gelu erf). Replaces the reference's fp32 products with
 * TF32 off (training/training_loop.py:504-505) that the bf16-piece kernels serve badly: the D heads' batch-folded
 * SpectralConv1d k = 1 / 9 products (reference networks/discriminator.py:39-42, :116-142), the decoder's narrow
 * 1x1 convolutions and GigaGAN projections of the 4^2 .. 8^2 blocks (networks/utils/convnext_utils.py:36-57,
 * :135-138, gigagan_utils.py:53-185), the adapter's 64-wide linears (ldm_utils.py:55-166) and the small FC layers
 * (networks/utils/shared.py FullyConnectedLayer). Layouts as vfm_gemm; contiguous extents and leading dims
 * multiples of 4 floats and 16-B aligned A / B (else VFM_NO_KERNEL). lgp > 0: the vfm_gemm_fold batch folding
 * (B[z] MN-contiguous [K][2^lgp], C[z] [M][2^lgp], N = batch 2^lgp). splits > 1 and / or reduce_batch (C = epi(
 * alpha sum_z A[z] B[z]), [M, N]): the virtual K-tiles (of every batch item when reduce_batch) cut into `splits`
 * chunks of fp32 partials in `workspace` (vfm_sgemm_workspace_floats), summed in a fixed order. tile: 0 128x128,
 * 1 128x64, 2 64x128, 3 64x64, < 0 chosen from the shape. */
int vfm_sgemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int batch,
              int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB, long long ldc,
              long long sC, float alpha, float beta, int bias_mode, int act, int lgp, float* workspace, int splits,
              int reduce_batch, int tile, void* stream);
long long vfm_sgemm_workspace_floats(int M, int N, int batch, int splits, int reduce_batch);

/* Large-tile form (csrc/gemm8.hip: 256 x 256 tiles, 4-phase LDS-DMA pipeline) of the same contract,
 * K % 64 == 0 (else VFM_NO_KERNEL). precision VFM_BF16: A / B are bf16 matrices as above. precision
 * VFM_F32 / VFM_F32X3: A / B hold the bf16 pieces of fp32 operands from vfm_split_f32 (3 pieces:
 * hi | mid | lo, or 2: hi | lo), stacked along K: K-contiguous [R][np K] (lda >= np K), MN-contiguous
 * [np K][R]; K is the fp32 depth, and the kernel accumulates the 6 (3) piece products of each
 * K-tile in fp32. Split-K: the virtual K-tiles of each output (terms x K/64, of every batch when
 * reduce_batch: C = sum_z A[z] B[z]) are cut into chunks of kchunk tiles (<= 0: no split); the
 * splits write fp32 partials to workspace (vfm_gemm8_workspace_floats floats) and a reduce pass
 * applies the epilogue in a fixed order. */
int vfm_gemm8(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype, int M, int N,
              int K, int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
              long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, float* workspace,
              int kchunk, int reduce_batch, void* stream);
/* vfm_gemm8 with explicit piece strides psA / psB (elements from piece 0 to piece 1 of an operand; 0 =
 * the stacked layouts above). Planar pieces [np][numel] of a whole fp32 tensor (vfm_split_f32 with R = 1,
 * K = numel) are addressed through any strided view of the tensor with the view's own lda / sA (in
 * elements, rows of K, not np K): one split of an activation serves its forward product and the
 * weight-gradient product of the backward, one split of a weight its forward and data-gradient
 * products (the fp32 1x1 convolutions and linears of reference networks/utils/convnext_utils.py:36-142,
 * ldm_utils.py:55-166 with TF32 off, training/training_loop.py:504-505). Same results as vfm_gemm8 on
 * the same pieces, bit for bit. */
int vfm_gemm8_pieces(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype, int M,
                     int N, int K, int batch, int a_kcont, long long lda, long long sA, long long psA, int b_kcont,
                     long long ldb, long long sB, long long psB, long long ldc, long long sC, float alpha,
                     float beta, int bias_mode, int act, float* workspace, int kchunk, int reduce_batch,
                     void* stream);
int vfm_gemm8_workspace_floats(int precision, int M, int N, int K, int batch, int kchunk,
                               int reduce_batch);  /* -1: too large */
/* bf16 form of the same contract on the LDS-DMA one-wave-per-SIMD kernel (csrc/gemm9.hip: 256 x 256 tiles,
 * 4 waves of 128 x 128, both operand tiles moved global -> LDS by LDS-DMA two K-tiles ahead, two barriers
 * per K-tile, accumulators pinned to AGPRs, C stored from the accumulators): the frozen SigLIP2 tower's
 * linears (reference networks/utils/vfms/siglip2_utils.py:120-121, HF SiglipMLP / SiglipAttention
 * projections under bf16 autocast) and the decoder's bf16 1x1 convolutions (reference
 * networks/utils/convnext_utils.py:135-138 pwconv1 / pwconv2, :241-249 the upsample's pointwise conv,
 * under autocast). bf16 A / B only; K % 64 == 0, N % 8 == 0, 16-B aligned A / B / C (else VFM_NO_KERNEL). */
int vfm_gemm9(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N, int K,
              int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
              long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, void* stream);
/* vfm_gemm9 with K splits and / or the batch reduction C = alpha sum_z A[z] B[z] (reduce_batch; C [M, N], row
 * stride ldc): the decoder's bf16 1x1 weight gradients dW = sum_b dY[b] X[b]^T (reference
 * networks/utils/convnext_utils.py:135-138, :241-249 under autocast; torch computes them as per-sample
 * fp32 products summed over the batch). S = min(splits, batch K / 64) chunks of the batch-concatenated
 * reduction write fp32 partials into `workspace` (vfm_gemm9_workspace_floats), combined in a fixed order
 * (deterministic). Plain products (no bias / activation); VFM_NO_KERNEL when not covered. */
int vfm_gemm9_ex(const void* A, const void* B, void* C, int out_dtype, int M, int N, int K, int batch, int a_kcont,
                 long long lda, long long sA, int b_kcont, long long ldb, long long sB, long long ldc, float alpha,
                 float* workspace, int splits, int reduce_batch, void* stream);
long long vfm_gemm9_workspace_floats(int M, int N, int K, int batch, int splits, int reduce_batch);
/* fp32 products on the same kernel with fp32-equivalent "f32x6" precision (the vfm_gemm8_pieces contract):
 * A / B are fp32 operands given as their three exact bf16 pieces (vfm_split_f32; psA / psB elements between
 * an operand's pieces, 0 = the stacked layouts along K), and the six piece products of order >= 2^-16 run as
 * consecutive virtual K-tiles into fp32 accumulators: C[z] (fp32) = alpha A[z] B[z] + bias. The decoder's
 * fp32 1x1 convolutions, the GigaGAN attention / FFN projections and the adapter linears (reference
 * networks/utils/convnext_utils.py:135-138, gigagan_utils.py:53-185, ldm_utils.py:55-166, fp32 with TF32 off:
 * training/training_loop.py:504-505). splits > 1 and / or reduce_batch (C = alpha sum_z A[z] B[z], [M, N]): whole real
 * K-tiles of the batch-concatenated reduction in S chunks of fp32 partials in `workspace`
 * (vfm_gemm9_workspace_floats), combined in a fixed order (no bias then). Beta 0, no activation;
 * VFM_NO_KERNEL when not covered. */
int vfm_gemm9_pieces(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int batch,
                     int a_kcont, long long lda, long long sA, long long psA, int b_kcont, long long ldb, long long sB,
                     long long psB, long long ldc, long long sC, float alpha, int bias_mode, float* workspace,
                     int splits, int reduce_batch, void* stream);
/* The ConvNeXt MLP's bf16 1x1 GEMMs on the persistent gemm9 kernel with the GELU in the epilogue (replaces
 * pwconv1 -> nn.GELU and the GELU backward of reference networks/utils/convnext_utils.py:135-142 under
 * autocast): C[z] = W[M, K] X[z][K, N] (W K-contiguous, lda; X N-contiguous, ldb, batch stride sB);
 * mode 1: C = h (may be null), C2 = g = bf16(GELU(bf16(h) s + b1)); mode 2: dg = bf16(acc),
 * dz = dg GELU'(h s + b1) with h read from H, C = dh = bf16(dz s), per-row partial sums of dz h (rsum0,
 * may be null) and dz (rsum1) at [batch][vfm_gemm9_gelu_parts(N)][M]. rscale [batch][M] (null: 1),
 * bias [M] (null: 0); C, C2, H share (ldc, sC). */
int vfm_gemm9_gelu(const void* W, const void* X, void* C, void* C2, const void* H, const float* rscale,
                   const float* bias, float* rsum0, float* rsum1, int mode, int M, int N, int K, int batch,
                   long long lda, long long ldb, long long sB, long long ldc, long long sC, void* stream);
int vfm_gemm9_gelu_parts(int N);
/* Kernel form of vfm_gemm9 (process-wide A/B switch for microbenchmarks): 1 = persistent (one workgroup per CU
 * walking the output tiles as one K-tile stream; default), 0 = one workgroup per output tile. Returns the
 * previous setting. */
int vfm_gemm9_set_mode(int persistent);
/* K-tile staging schedule of vfm_gemm8 / vfm_gemm8_gelu (process-wide A/B switch for microbenchmarks):
 * 1 = half-tile slots restaged two K-tiles ahead, 0 = one K-tile ahead (default). Returns the previous
 * setting. */
int vfm_gemm8_set_schedule(int deep);
/* The ConvNeXt MLP's bf16 1x1 GEMMs with their GELU fused into the epilogue (replaces the
 * pwconv1 -> nn.GELU and the GELU backward of reference networks/utils/convnext_utils.py:135-142
 * around torch's batched matmul): C[z] = W X[z], W [M, K] K-contiguous (row stride lda), X[z]
 * [K, N] N-contiguous (row stride ldb, batch stride sB); C, C2, H: [batch][M][N] (ldc, sC).
 *   mode 1: C = h = bf16(W X) (C may be null), C2 = g = bf16(GELU(h * rscale[z][m] + bias[m]));
 *   mode 2: acc = dg: dz = bf16(dg) * GELU'(H * s + b), C = dh = bf16(dz * s); per-row partial
 *           sums of dz * H (rsum0, may be null) and dz (rsum1) at [z][p][m], p < vfm_gemm8_gelu_parts(N).
 * GELU is the exact-erf form. K % 64, N % 8 and the strides % 8 == 0, else VFM_NO_KERNEL. */
int vfm_gemm8_gelu(const void* W, const void* X, void* C, void* C2, const void* H, const float* rscale,
                   const float* bias, float* rsum0, float* rsum1, int mode, int M, int N, int K, int batch,
                   long long lda, long long ldb, long long sB, long long ldc, long long sC, void* stream);
int vfm_gemm8_gelu_parts(int N);
/* Microbenchmarks only: a device buffer of 16 int64 per launched block that the following gemm8
 * launches fill with s_memrealtime (100 MHz) stamps (entry, first K-tile landed, then per tile: main loop done,
 * epilogue done); NULL (the default) turns them off. */
int vfm_gemm8_set_stamps(long long* buf);
/* fp32 -> bf16 pieces of one GEMM operand along its reduction dimension K (precision VFM_F32: 3
 * pieces hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid), x = hi + mid + lo exactly;
 * VFM_F32X3: 2 pieces hi, lo). kcont = 1: src [R][K] (row stride ld) -> dst [R][np K];
 * kcont = 0: src [K][R] -> dst [np K][R]; batch strides sb (src) / db (dst) in elements. */
int vfm_split_f32(const float* src, void* dst, int R, int K, long long ld, long long sb, long long db, int batch,
                  int precision, int kcont, void* stream);

/* ---------------------------------------------------------------------------
 * Discrete latent: codebook lookup of VectorQuantizer (replaces the
 * `torch.argmax(F.normalize(f) @ F.normalize(codebook).T, dim=1)` of
 * networks/utils/quant_utils.py:84-86 and f_to_idx :126-131).
 *   features: fp32 [N, C], row stride `ld` elements (>= C; unit column stride).
 *   codebook: fp32 [V, C] contiguous (raw weights; normalised inside).
 *   indices : int64 [N] output = first index of the maximal cosine (NaN = maximal).
 * Fixed fp32 evaluation order (left-to-right sums, no FMA contraction, IEEE sqrt and
 * division), so results are bit-reproducible against oracle/ops_oracle.c.
 * C in {1, 2, 3, 4, 8, 16, 32, 64}; other widths return VFM_NO_KERNEL. */
int vfm_codebook_argmax(const float* features, long long ld, const float* codebook, int N, int C, int V,
                        long long* indices, void* stream);

/* ---------------------------------------------------------------------------
 * ConvNeXt MLP channel GEMM with the GELU fused into its epilogue (replaces the
 * modulated 1x1 conv + GELU of convnext_utils.py:135-138, and in backward the
 * 4C->C conv's data gradient + GELU backward). bf16 operands, fp32 accumulation.
 *   A: bf16 [M, K] row-major (W1 [4C, C]; backward: W2^T [4C, C]);
 *   X: bf16 [B, K, N] (forward: the GroupNorm output m; backward: dy);
 *   scale: fp32 [B, M] demodulation (NULL = 1); bias: fp32 [M] (NULL = 0).
 *   mode 0: out0 = bf16(A.X) (NULL: not written), out1 = bf16(GELU(out0 * scale + bias)).
 *   mode 1: dg = bf16(A.X), z = h * scale + bias (h: bf16 [B, M, N]), dz = dg * GELU'(z);
 *           out0 = bf16(dz * scale); part0 / part1: fp32 [B, tiles, M] per-tile sums over N of
 *           dz * h and dz over 64-column tiles (tiles = vfm_pw_gemm_gelu_tiles(N) = N / 64), reduced by
 *           the caller.
 * K in {128, 256, 512}, M % 128 == 0, M <= 2048, N % 128 == 0 (else VFM_NO_KERNEL). */
int vfm_pw_gemm_gelu(const void* A, const void* X, const float* scale, const float* bias, const void* h,
                     void* out0, void* out1, float* part0, float* part1, int mode, int B, int M, int K, int N,
                     void* stream);
int vfm_pw_gemm_gelu_tiles(int N);

/* The whole ConvNeXt MLP of convnext_utils.py:135-142 without autograd (the D phase's
 * no-grad generator pass), bf16 in/out, fp32 accumulation, hidden tensor kept on chip:
 *   out = x_in + gamma * (bf16(W2 . g) + b2),  g = bf16(GELU(bf16(W1 . m) * s + b1)).
 *   W1: bf16 [4C, C]; m, x_in, out: bf16 [B, C, N]; s: fp32 [B, 4C] (NULL = 1);
 *   b1: fp32 [4C]; W2: bf16 [C, 4C]; b2, gamma: fp32 [C] (NULL = 0 / 1).
 *   hout, gout: bf16 [B, 4C, N] (both or neither; NULL: not written) = bf16(W1 . m) and g,
 *   yout: bf16 [B, C, N] (NULL: not written) = bf16(W2 . g) — what the backward needs.
 * C in {128, 256}, N % 128 == 0 (else VFM_NO_KERNEL). */
int vfm_convnext_mlp_fwd(const void* W1, const void* m, const float* s, const float* b1, const void* W2,
                         const float* b2, const float* gamma, const void* xin, void* out, void* hout, void* gout,
                         void* yout, int B, int C, int N, void* stream);

/* ---------------------------------------------------------------------------
 * LPIPS distance head (replaces the per-tap tail of training/lpips.py LPIPS.forward:
 * `(normalize_tensor(f0) - normalize_tensor(f1)) ** 2` -> `lin` 1x1 conv C->1 (no bias);
 * the `spatial_average` stays a mean over r in the caller).
 *   f0, f1: fp32 [B, C, HW] contiguous (NCHW VGG16 taps); w: fp32 [C] (lin weight).
 *   fwd writes r [B, HW] and the channel norms n0, n1 [B, HW] (saved for backward).
 *   bwd: gs fp32 [B] = upstream gradient of each r[b, :]; writes g0 and/or g1 [B, C, HW]
 *   (either may be NULL). */
int vfm_lpips_head_fwd(const float* f0, const float* f1, const float* w, float* r, float* n0, float* n1,
                       int B, int C, long long HW, void* stream);
int vfm_lpips_head_bwd(const float* f0, const float* f1, const float* w, const float* n0, const float* n1,
                       const float* gs, float* g0, float* g1, int B, int C, long long HW, void* stream);
/* Same head on NHWC (channels_last) taps [B, HW, C], C in {64, 128, 256, 512} (the HIP VGG16
 * stack's layout; 16-B aligned); r / n0 / n1 / gs as above, g0 / g1 NHWC. */
int vfm_lpips_head_fwd_nhwc(const float* f0, const float* f1, const float* w, float* r, float* n0, float* n1,
                            int B, int C, long long HW, void* stream);
int vfm_lpips_head_bwd_nhwc(const float* f0, const float* f1, const float* w, const float* n0, const float* n1,
                            const float* gs, float* g0, float* g1, int B, int C, long long HW, void* stream);

/* Depthwise K x K conv (K in {3, 5, 7}, pad (K-1)/2, stride 1) of bf16 NCHW planes on the MFMA
 * cores (banded-matrix form, csrc/dwconv_mfma.hip); same contract as vfm_dwconv2d_fwd (noise: fp32
 * [H, W] added to every channel, or NULL), taps w fp32 [C, K, K] rounded to bf16 (the reference's
 * autocast conv: replaces convnext_utils.py:121-124 / :243 nn.Conv2d(groups=C) for the bf16 blocks,
 * and its data gradient with the rotated taps). res: bf16 [B, C, H, W] added to the fp32 result before
 * the output rounding (the residual branch's gradient of the same input), or NULL. W % 16 == 0,
 * 16-B aligned x / y / noise / res; VFM_NO_KERNEL otherwise. */
int vfm_dwconv2d_fwd_mfma(const void* x, const float* w, const float* bias, const float* noise, const void* res,
                          void* y, int B, int C, int H, int W, int K, int pad, void* stream);
/* The same convs with the taps read rotated by 180 degrees when flip != 0: the data gradient
 * (dx = dwconv(dy, rot180(w)), pad' = K - 1 - pad) without a flipped copy of the weights. */
int vfm_dwconv2d_fwd_ex(const void* x, const float* w, const float* bias, const float* noise, void* y, int dtype,
                        int B, int C, int H, int W, int K, int pad, int flip, void* stream);
/* vfm_dwconv2d_fwd_ex + res (a tensor of y's shape and dtype, or null) added to y in the store: the ConvNeXt
 * layer's residual-branch gradient summed into the data gradient of the fp32 planes' dwconv (reference
 * networks/utils/convnext_utils.py:117-142, x feeding both the dwconv and the residual). */
int vfm_dwconv2d_fwd_res(const void* x, const float* w, const float* bias, const float* noise, const void* res,
                         void* y, int dtype, int B, int C, int H, int W, int K, int pad, int flip, void* stream);
int vfm_dwconv2d_fwd_mfma_ex(const void* x, const float* w, const float* bias, const float* noise, const void* res,
                             void* y, int B, int C, int H, int W, int K, int pad, int flip, void* stream);
/* vfm_dwconv2d_fwd_mfma_ex that also writes, when npart is given (with nplane fp32 [H, W], 16-B aligned),
 * npart[u] = wave u's share of sum_{b,c,y,x} x[b,c,y,x] nplane[y,x] for u < vfm_dwconv2d_fwd_mfma_units(...):
 * in the data-gradient call (x = dY) the gradient of the legacy noise strength (reference
 * convnext_utils.py noise_const * noise_strength added after the dwconv) without another pass over dY. */
int vfm_dwconv2d_fwd_mfma_nz(const void* x, const float* w, const float* bias, const float* noise, const void* res,
                             void* y, const float* nplane, float* npart, int B, int C, int H, int W, int K, int pad,
                             int flip, void* stream);
long long vfm_dwconv2d_fwd_mfma_units(int B, int C, int H, int W, int K, int pad);
/* vfm_dwconv2d_fwd_mfma (no residual, no flip) that also writes the GroupNorm statistics of the
 * bf16-rounded y: gstat [units][4] (16-B aligned, units = vfm_dwconv2d_fwd_mfma_units(...)) =
 * {count, shift, sum (y - shift), sum (y - shift)^2} per wave, the units of one (sample, channel)
 * plane consecutive. Replaces the statistics pass of the GroupNorm that follows the ConvNeXt
 * block's dwconv (reference convnext_utils.py:117-127 dwconv -> norm), see vfm_group_norm_fwd_stats. */
int vfm_dwconv2d_fwd_mfma_gs(const void* x, const float* w, const float* bias, const float* noise, void* y,
                             float* gstat, int B, int C, int H, int W, int K, int pad, void* stream);
/* dw[c, t] = sum_r partial[r, c, t] (t < KK), db[c] = sum_r partial[r, c, KK] over the [rows, C, KK + 1]
 * partials of the depthwise weight-gradient kernels (either output may be null). */
int vfm_dwconv2d_wgrad_reduce(const float* partial, float* dw, float* db, int rows, int C, int KK, void* stream);
/* Weight (and bias) gradient of the same conv on MFMA: partial[t, c, 0 .. K*K-1] = per-wave sums of
 * dW[c][ky][kx] = sum dy[b,c,y,x] x[b,c,y+ky-pad,x+kx-pad], partial[t, c, K*K] = sum dy; t < tiles
 * = vfm_dwconv2d_bwd_weight_mfma_tiles(...) (same partial layout as vfm_dwconv2d_bwd_weight; the
 * caller sums over t in a fixed order). bf16 x / dy, W % 16 == 0. */
int vfm_dwconv2d_bwd_weight_mfma_tiles(int B, int C, int H, int W, int K, int pad);
int vfm_dwconv2d_bwd_weight_mfma(const void* x, const void* dy, float* partial, int B, int C, int H, int W, int K,
                                 int pad, void* stream);

/* ---- ToRGB: modulated 1x1 (no demodulation) to O <= 4 image channels ----------------------
 * Replaces networks/utils/convnext_utils.py:145-187 (ConvNeXtToRGBLayer.forward: x * style, 1x1
 * conv, + bias) in both directions as one HBM pass.
 *   x: [B, C, P] (dtype VFM_F32 / VFM_BF16, P % 8 == 0, 16-B aligned); wm: fp32 [B, O, C] =
 *   weight[o, c] * style[b, c]; bias fp32 [O]; y fp32 [B, O, P] = round_x(sum_c wm x) + bias
 *   (round_x: to bf16 when x is bf16, the reference's bf16 product before the fp32 bias).
 * bwd: dy fp32 [B, O, P] -> dx [B, C, P] (x's dtype) = sum_o wm dy, and per pixel split s the
 *   partial tpart[b, s, o, c] = sum_{p in split s} x[b, c, p] dy[b, o, p] (C % 16 == 0;
 *   S from vfm_torgb_bwd_splits; tpart holds B * S * O * C floats). */
int vfm_torgb_fwd(const void* x, const float* wm, const float* bias, float* y, int dtype, int B, int O, int C,
                  int P, void* stream);
int vfm_torgb_bwd_splits(int B, int C, int P);
int vfm_torgb_bwd(const void* x, const float* dy, const float* wm, void* dx, float* tpart, int dtype, int B, int O,
                  int C, int P, int S, void* stream);

/* ---- Latent posterior (replaces networks/utils/kl_utils.py:30-56 DiagonalGaussianDistribution's
 * sample() and kl() on the continuous latent): params fp32 [B, 2C, P] (mean | logvar channels),
 * eps fp32 [B, C, P] (drawn by the caller as the reference does); z = mean + exp(clamp(logvar,
 * -30, 20) / 2) eps, kl[b] = 0.5 sum_{c,p}(mean^2 + exp(lv) - 1 - lv) (z or kl may be NULL).
 * bwd: dz [B, C, P] and dkl [B] (either may be NULL) -> dparams [B, 2C, P]. Deterministic. */
int vfm_posterior_fwd(const float* params, const float* eps, float* z, float* kl, int B, int C, long long P,
                      void* stream);
int vfm_posterior_bwd(const float* params, const float* eps, const float* dz, const float* dkl, float* dparams,
                      int B, int C, long long P, void* stream);

/* ---- BatchNormLocal (1-d) + LeakyReLU of the projected discriminator's heads (replaces
 * networks/discriminator.py:45-71 + the head blocks' nn.LeakyReLU(0.2), :102-109): x fp32 [B, C, L] in
 * G virtual batches (B % G == 0), statistics per (group, channel) over the group's samples and L;
 * y = lrelu((x - mean) rstd w + b, slope), mean / rstd [G, C] saved. bwd: dx and part [2, G, C] =
 * per-group (sum dz xhat, sum dz) for dw / db (the caller sums over G). w / b may be NULL. */
int vfm_bnl1d_lrelu_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd, int B,
                        int C, int L, int G, float eps, float slope, void* stream);
int vfm_bnl1d_lrelu_bwd(const float* x, const float* dy, const float* w, const float* b, const float* mean,
                        const float* rstd, float* dx, float* part, int B, int C, int L, int G, float slope,
                        void* stream);

/* ---- Multi-scale PatchGAN (stage 3), fp32 NHWC ----------------------------------------------
 * Replace networks/discriminator.py:180-228 (NLayerDiscriminator's nn.Conv2d k4 s2/s1 p2 layers,
 * run by the reference on cuDNN) around our MFMA GEMM, and :75-99 (BatchNormLocal2d) + LeakyReLU.
 * im2col: A[m, (ky k + kx) C + c] = x[b, s oy - pad + ky, s ox - pad + kx, c] (0 outside), m =
 *   (b Ho + oy) Wo + ox, x NHWC [B, H, W, C], A row stride ldA >= k k C.
 * col2im: dX[b, iy, ix, c] = sum of dA[m, tap C + c] over the taps that read (iy, ix); with dy1
 *   ([M]) and w1 ([k k C]) instead of dA: dA[m, j] = dy1[m] w1[j] (the 1-channel layer).
 * rowdot: y[m] = sum_k A[m, k] w[k] (+ bias[0]); coldot: part[s, k] = sum_{m in split s} A[m, k] v[m]
 *   (S from vfm_coldot_splits; part holds S * K floats).
 * bnl_lrelu: x NHWC [B, P = H W, C] in G virtual batches of B / G samples; per (g, c) mean / rstd
 *   over (samples, P); y = lrelu((x - mean) rstd w + b, slope) (w / b may be NULL); bwd writes dx
 *   and dw / db (summed over groups; may be NULL). C % 4 == 0 and 256 % (C / 4) == 0; ws holds
 *   vfm_bnl_workspace_floats floats; deterministic (fixed-order partial sums). */
int vfm_im2col_nhwc_f32(const float* x, float* A, long long ldA, int B, int H, int W, int C, int Ho, int Wo, int k,
                        int stride, int pad, void* stream);
int vfm_col2im_nhwc_f32(const float* dA, long long ldA, const float* dy1, const float* w1, float* dX, int B, int H,
                        int W, int C, int Ho, int Wo, int k, int stride, int pad, void* stream);
int vfm_rowdot_f32(const float* A, long long ldA, const float* w, const float* bias, float* y, int M, int K,
                   void* stream);
int vfm_coldot_splits(int M, int K);
int vfm_coldot_f32(const float* A, long long ldA, const float* v, float* part, int M, int K, int S, void* stream);
long long vfm_bnl_workspace_floats(int B, int P, int C, int G);
int vfm_bnl_lrelu_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd, float* ws,
                      int B, int P, int C, int G, float eps, float slope, void* stream);
int vfm_bnl_lrelu_bwd(const float* x, const float* dy, const float* w, const float* b, const float* mean,
                      const float* rstd, float* dx, float* dw, float* db, float* ws, int B, int P, int C, int G,
                      float slope, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VFMVAE_H */
