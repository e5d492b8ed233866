/*
 * ops_oracle.c — CPU oracle for the StyleGAN-lineage ops of the VFM-VAE hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product path links or calls this file;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may.
 *
 * Plain-C, double-precision restatements written straight from the reference's
 * definitions (not from its kernels):
 *   oracle_upfirdn2d      <- torch_utils/ops/upfirdn2d.py:166-211 (_upfirdn2d_ref):
 *                            zero-insert `up`, pad/crop, correlate with the flipped
 *                            filter (convolution), keep every `down`-th sample, gain.
 *   oracle_bias_act       <- torch_utils/ops/bias_act.py:21-31 (activation table) and
 *                            :90-120 (_bias_act_ref).
 *   oracle_filtered_lrelu <- torch_utils/ops/filtered_lrelu.py:120-153 (_filtered_lrelu_ref)
 *                            plus the 2-bit sign codes of filtered_lrelu.cu:1105-1160
 *                            (bit0 = negative branch taken, code 2 = clamped).
 *   oracle_codebook_argmax <- networks/utils/quant_utils.py:84-86 and :126-131
 *                            (F.normalize(f) @ F.normalize(codebook).T -> argmax), fp32,
 *                            in the fixed evaluation order the HIP kernel uses
 *                            (left-to-right rounded squares, IEEE sqrt/division, dot
 *                            product as a left-to-right FMA chain = torch's CPU order).
 * Parity pin: tests/test_oracle_ops.py checks these against golden vectors generated
 * from the reference itself (tests/golden/make_golden_ops.py, make_golden_vq.py).
 * Layout: all arrays dense NCHW.
 */
/* Built with -ffp-contract=off (oracle/Makefile): no fused multiply-adds anywhere. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* u(j) of the zero-inserted signal along one axis: index into x or -1 if zero. */
static int upsampled_index(int j, int up, int size) {
    if (j < 0 || j % up != 0) return -1;
    int i = j / up;
    return i < size ? i : -1;
}

void oracle_upfirdn2d(const double* x, int N, int C, int H, int W,
                      const double* f, int fh, int fw,
                      int upx, int upy, int downx, int downy,
                      int px0, int py0, int flip, double gain,
                      double* y, int outH, int outW) {
    for (int nc = 0; nc < N * C; ++nc) {
        const double* xp = x + (long)nc * H * W;
        double* yp = y + (long)nc * outH * outW;
        for (int oy = 0; oy < outH; ++oy)
            for (int ox = 0; ox < outW; ++ox) {
                double acc = 0.0;
                for (int ty = 0; ty < fh; ++ty) {
                    int iy = upsampled_index(oy * downy + ty - py0, upy, H);
                    if (iy < 0) continue;
                    for (int tx = 0; tx < fw; ++tx) {
                        int ix = upsampled_index(ox * downx + tx - px0, upx, W);
                        if (ix < 0) continue;
                        /* conv2d correlates with flip(f) unless flip (correlation) requested */
                        int fy = flip ? ty : fh - 1 - ty;
                        int fx = flip ? tx : fw - 1 - tx;
                        acc += f[fy * fw + fx] * xp[iy * W + ix];
                    }
                }
                yp[oy * outW + ox] = acc * gain;
            }
    }
}

static double act_fn(int act, double v, double alpha) {
    switch (act) {
    case 1: return v;                                            /* linear */
    case 2: return v > 0 ? v : 0.0;                              /* relu */
    case 3: return v > 0 ? v : v * alpha;                        /* lrelu */
    case 4: return tanh(v);                                      /* tanh */
    case 5: return 1.0 / (1.0 + exp(-v));                        /* sigmoid */
    case 6: return v > 0 ? v : expm1(v);                         /* elu (alpha 1) */
    case 7: {                                                    /* selu */
        const double s = 1.0507009873554804934193349852946, a = 1.6732632423543772848170429916717;
        return v > 0 ? s * v : s * a * expm1(v);
    }
    case 8: return v > 20.0 ? v : log1p(exp(v));                 /* softplus (torch threshold 20) */
    case 9: return v / (1.0 + exp(-v));                          /* swish */
    }
    return NAN;
}

/* y[i] = clamp(act(x[i] + b[(i / stepB) % sizeB]) * gain); clamp < 0 disables. */
void oracle_bias_act(const double* x, const double* b, long long numel, long long stepB, int sizeB,
                     int act, double alpha, double gain, double clamp, double* y) {
    for (long long i = 0; i < numel; ++i) {
        double v = x[i];
        if (b) v += b[(i / stepB) % sizeB];
        v = act_fn(act, v, alpha) * gain;
        if (clamp >= 0) v = v < -clamp ? -clamp : (v > clamp ? clamp : v);
        y[i] = v;
    }
}

/*
 * filtered_lrelu: returns y [N,C,outH,outW] and the unpacked sign code of every
 * intermediate element codes [N,C,ch,cw] (0, 1 = negative, 2 = clamped).
 * The intermediate is upfirdn2d(x + b, fu, up, pad, gain=up^2) of size ch x cw.
 */
void oracle_filtered_lrelu(const double* x, const double* b, int N, int C, int H, int W,
                           const double* fu, int fuh, int fuw, const double* fd, int fdh, int fdw,
                           int up, int down, int px0, int px1, int py0, int py1,
                           double gain, double slope, double clamp, int flip,
                           double* y, int outH, int outW, unsigned char* codes, int ch, int cw) {
    (void)px1; (void)py1;
    long plane = (long)H * W;
    double* xb = (double*)malloc(sizeof(double) * N * C * plane);
    double* mid = (double*)malloc(sizeof(double) * N * C * (long)ch * cw);
    for (int nc = 0; nc < N * C; ++nc)
        for (long i = 0; i < plane; ++i) xb[nc * plane + i] = x[nc * plane + i] + (b ? b[nc % C] : 0.0);
    oracle_upfirdn2d(xb, N, C, H, W, fu, fuh, fuw, up, up, 1, 1, px0, py0, flip, (double)(up * up), mid, ch, cw);
    for (long i = 0; i < (long)N * C * ch * cw; ++i) {
        double v = mid[i] * gain;
        unsigned char s = 0;
        if (v < 0) { v *= slope; s = 1; }
        if (fabs(v) > clamp) { v = v < 0 ? -clamp : clamp; s = 2; }
        mid[i] = v;
        if (codes) codes[i] = s;
    }
    oracle_upfirdn2d(mid, N, C, ch, cw, fd, fdh, fdw, 1, 1, down, down, 0, 0, flip, 1.0, y, outH, outW);
    free(xb);
    free(mid);
}

/* ------------------------------------------------------------------------------------------
 * Codebook lookup (fp32 on purpose: the indices must match the fp32 reference bit for bit).
 * F.normalize(x, dim=-1) = x / clamp_min(||x||_2, 1e-12)  (torch.nn.functional.normalize);
 * score = <f_hat, w_hat>, idx = first maximal index, NaN counts as maximal (torch.argmax). */
static void vq_normalize(const float* x, int C, float* o) {
    float s = x[0] * x[0];
    for (int i = 1; i < C; ++i) s = s + x[i] * x[i];
    float n = sqrtf(s);
    n = n < 1e-12f ? 1e-12f : n;
    for (int i = 0; i < C; ++i) o[i] = x[i] / n;
}

void oracle_codebook_argmax(const float* f, long long ld, const float* w, int N, int C, int V, long long* idx) {
    float* wn = (float*)malloc(sizeof(float) * (size_t)V * C);
    float* fn = (float*)malloc(sizeof(float) * (size_t)C);
    for (int v = 0; v < V; ++v) vq_normalize(w + (size_t)v * C, C, wn + (size_t)v * C);
    for (int n = 0; n < N; ++n) {
        vq_normalize(f + (size_t)n * ld, C, fn);
        float best = -INFINITY;
        long long bi = 0;
        for (int v = 0; v < V; ++v) {
            const float* cw = wn + (size_t)v * C;
            float d = fn[0] * cw[0];
            for (int i = 1; i < C; ++i) d = fmaf(fn[i], cw[i], d);   /* FMA chain, as torch's CPU sgemm */
            if (d > best) {
                best = d;
                bi = v;
            } else if (isnan(d)) {
                bi = v;
                break;
            }
        }
        idx[n] = bi;
    }
    free(wn);
    free(fn);
}
