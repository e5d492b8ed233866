// One launch for a phase's whole optimizer step: Adam over every parameter that has a gradient (reference
// training/training_loop.py:722-732, torch.optim.Adam with the config's betas / eps / lr) and, in the G phase,
// the G_ema update of the same parameters (reference :734-742, p_ema <- p.lerp(p_ema, beta)) on the freshly
// stepped values -- instead of torch's multi-tensor Adam (a launch per ~100 tensors) followed by a second
// multi-tensor pass that re-reads every parameter for the lerp.
//
// Work list: a device table of tensors (AdamT) and one of chunks (tensor, chunk index) of CH elements; one block
// per chunk. The tables depend only on the storage of the parameters, gradients (views of the phase's flat
// gradient buffer), moment buffers and EMA copies, which persist across steps, so the host builds and uploads
// them once per parameter set (torch_utils/ops/adam_hip.py) and a step is one launch with scalar arguments.
//
// Arithmetic: the expression forms and precisions of torch's fused Adam (ATen fused_adam_utils.cuh, ORIGINAL
// mode, no amsgrad / maximize / grad scaling): the moments in double from float operands, rounded to float on
// store; step_size = lr / bc1 and the denominator rounded to float; the update in float; bc1 = 1 - beta1^step,
// sqrt(1 - beta2^step) from the host in double. The lerp is torch's (|w| < 0.5: self + w (end - self), else
// end - (end - self) (1 - w)) in float. Per element: 28 B (p, g, m, v read; p, m, v written), + 8 B with EMA.
//
// Raw gradients (vfm_adam_ema_step_raw): at world size 1 the phase's gradients are the tensors autograd allocated
// this step (training_loop.FlatGradSync direct mode: no per-parameter hooks, no gather into a flat buffer), so
// their addresses come per step in a device array, and the kernel applies what FlatGradSync.finish() applies to
// the flat buffer -- g * gain in float, then nan_to_num(nan 0, +inf 1e5, -inf -1e5) -- as it reads them.
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int THREADS = 256, CH = 8192;

struct AdamT {                  // 64 B, the host writes it as 8 int64 (torch_utils/ops/adam_hip.py)
    float* p;
    const float* g;
    float* m;
    float* v;
    float* e;                   // EMA copy (null: none)
    long long n;
    long long vec;              // every pointer 16-B aligned and n % 4 == 0
    float* step;                // the optimizer's fp32 step counter of this tensor (null: the host advances it)
};

struct AdamHyper {
    double lr, beta1, beta2, wd, eps, bc1, bc2_sqrt;
    float ema_w;
    int has_wd;
    float gscale;               // raw gradients: g * gscale, then nan_to_num
    int clean;
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamHyper& h) {
    if (h.clean) {
        g *= h.gscale;
        g = isnan(g) ? 0.f : isinf(g) ? (g > 0.f ? 1e5f : -1e5f) : g;
    }
    if (h.has_wd) g = (float)((double)g + (double)p * h.wd);
    m = (float)(h.beta1 * (double)m + (1.0 - h.beta1) * (double)g);
    v = (float)(h.beta2 * (double)v + (1.0 - h.beta2) * (double)g * (double)g);
    const float step_size = (float)(h.lr / h.bc1);
    const float denom = (float)((double)sqrtf(v) / h.bc2_sqrt + h.eps);
    p -= step_size * m / denom;
}

__device__ __forceinline__ float lerp1(float self, float end, float w) {
    return fabsf(w) < 0.5f ? self + w * (end - self) : end - (end - self) * (1.f - w);
}

__global__ __launch_bounds__(THREADS) void adam_ema_kernel(const AdamT* __restrict__ T, const int2* __restrict__ chunks,
                                                           const float* const* __restrict__ graw, AdamHyper h) {
    const int2 c = chunks[blockIdx.x];
    AdamT t = T[c.x];
    if (t.step && c.y == 0 && threadIdx.x == 0) *t.step += 1.f;     // torch's _foreach_add_(steps, 1)
    if (graw) {                 // this step's gradient of tensor c.x (its record's vec flag covers p, m, v, e and n)
        t.g = graw[c.x];
        t.vec = t.vec && (reinterpret_cast<unsigned long long>(t.g) & 15) == 0;
    }
    const long long s = (long long)c.y * CH, e = min(t.n, s + (long long)CH);
    if (t.vec) {
        for (long long i = s + 4LL * threadIdx.x; i < e; i += 4LL * THREADS) {
            float4 p = *reinterpret_cast<const float4*>(t.p + i);
            const float4 g = *reinterpret_cast<const float4*>(t.g + i);
            float4 m = *reinterpret_cast<const float4*>(t.m + i);
            float4 v = *reinterpret_cast<const float4*>(t.v + i);
            adam1(p.x, g.x, m.x, v.x, h);
            adam1(p.y, g.y, m.y, v.y, h);
            adam1(p.z, g.z, m.z, v.z, h);
            adam1(p.w, g.w, m.w, v.w, h);
            *reinterpret_cast<float4*>(t.p + i) = p;
            *reinterpret_cast<float4*>(t.m + i) = m;
            *reinterpret_cast<float4*>(t.v + i) = v;
            if (t.e) {
                float4 q = *reinterpret_cast<const float4*>(t.e + i);
                q.x = lerp1(q.x, p.x, h.ema_w);
                q.y = lerp1(q.y, p.y, h.ema_w);
                q.z = lerp1(q.z, p.z, h.ema_w);
                q.w = lerp1(q.w, p.w, h.ema_w);
                *reinterpret_cast<float4*>(t.e + i) = q;
            }
        }
    } else {
        for (long long i = s + threadIdx.x; i < e; i += THREADS) {
            float p = t.p[i], m = t.m[i], v = t.v[i];
            adam1(p, t.g[i], m, v, h);
            t.p[i] = p;
            t.m[i] = m;
            t.v[i] = v;
            if (t.e) t.e[i] = lerp1(t.e[i], p, h.ema_w);
        }
    }
}

}  // namespace

// Elements per chunk of the work list (the host splits every tensor into ceil(n / CH) chunks). A record's step
// pointer (its last 8 B; null: none) names the optimizer's fp32 step counter of that tensor, advanced by 1 in the
// launch (the host's bc1 / bc2_sqrt are for the advanced count).
extern "C" int vfm_adam_chunk_elems(void) { return CH; }

// One Adam (+ EMA) step over the tensors of `tensors` (device array of ntensors 64-B records: p, g, m, v, ema or
// null, n, vec flag, 0) through the chunk list `chunks` (device array of nchunks (tensor, chunk) int pairs).
// bc1 = 1 - beta1^step, bc2_sqrt = sqrt(1 - beta2^step); ema_w: the lerp weight 1 - beta_ema (records with a
// null ema pointer ignore it).
extern "C" int vfm_adam_ema_step_raw(const void* tensors, int ntensors, const void* chunks, int nchunks,
                                     const void* grads, float gscale, int clean, double lr, double beta1, double beta2,
                                     double weight_decay, double eps, double bc1, double bc2_sqrt, float ema_w,
                                     void* stream);

extern "C" int vfm_adam_ema_step(const void* tensors, int ntensors, const void* chunks, int nchunks, double lr,
                                 double beta1, double beta2, double weight_decay, double eps, double bc1,
                                 double bc2_sqrt, float ema_w, void* stream) {
    return vfm_adam_ema_step_raw(tensors, ntensors, chunks, nchunks, nullptr, 1.f, 0, lr, beta1, beta2, weight_decay,
                                 eps, bc1, bc2_sqrt, ema_w, stream);
}

// vfm_adam_ema_step with the gradients read through `grads` (device array of ntensors float pointers, one per record,
// replacing the records' g; null: use the records' g) and, when clean != 0, transformed to nan_to_num(g * gscale)
// (nan 0, +inf 1e5, -inf -1e5) before use. Each gradient holds its tensor's n contiguous floats.
extern "C" int vfm_adam_ema_step_raw(const void* tensors, int ntensors, const void* chunks, int nchunks,
                                     const void* grads, float gscale, int clean, double lr, double beta1, double beta2,
                                     double weight_decay, double eps, double bc1, double bc2_sqrt, float ema_w,
                                     void* stream) {
    if (!tensors || !chunks || ntensors <= 0 || nchunks < 0 || !(bc1 > 0.0) || !(bc2_sqrt > 0.0)) return VFM_ERR_ARGS;
    if (nchunks == 0) return 0;
    AdamHyper h{lr, beta1, beta2, weight_decay, eps, bc1, bc2_sqrt, ema_w, weight_decay != 0.0, gscale, clean != 0};
    VFM_LAUNCH(adam_ema_kernel, dim3((unsigned)nchunks), dim3(THREADS), 0, (hipStream_t)stream,
               (const AdamT*)tensors, (const int2*)chunks, (const float* const*)grads, h);
    return launch_status();
}
