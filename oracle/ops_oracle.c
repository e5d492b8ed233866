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
 * Parity pin: tests/test_oracle_ops.py checks these against golden vectors generated
 * from the reference itself (tests/golden/make_golden_ops.py).
 * Layout: all arrays dense NCHW.
 */
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
