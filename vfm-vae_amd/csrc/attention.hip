// Fused multi-head self-attention forward (flash-style), bf16 in/out, fp32 softmax.
//
// Replaces `F.scaled_dot_product_attention(q, k, v)` inside the frozen ViT towers
// (HF SiglipAttention under bf16 autocast, reference networks/utils/vfms/siglip2_utils.py:121;
// DINOv2 / CLIP towers of configs 0 and 3): O = softmax(Q K^T * scale) V per (batch, head),
// head dim 64, any token count N, no mask, no dropout. Forward only: the towers run frozen
// under no_grad.
//
// Layout: Q, K, V, O are [B, N, H, 64] views with element strides (batch, token, head) and
// unit stride along the head dim. The SigLIP tower passes its packed
// qkv GEMM output [B, N, 3, H, 64] directly (stride_n = 3*H*64), so no q/k/v split or
// transpose copies are made, and O lands in the [B, N, H*64] layout the output projection
// reads.
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md App. B "Fused attention prefill"):
//   * workgroup = 4 waves = 128 query rows of one (b, h); wave = 32 query rows;
//   * per 64-key tile, K and V are staged in LDS (128-B rows, 16-B chunks XOR-swizzled by
//     (key>>1)&7 so the 32-row ds_read_b128 of K and the ds_read_b64_tr_b16 of V are
//     conflict-free), the next tile's global loads issued before the current tile's math
//     (register staging, written to LDS after the barrier);
//   * swapped QK^T: S^T = K . Q^T with v_mfma_f32_32x32x16_bf16 puts one query per lane
//     (column) and its keys in the 16 accumulator registers, so the row max / row sum are
//     lane-local plus one exchange with lane^32;
//   * O^T = V^T . P^T: the bf16-converted S^T registers ARE the B operand (accumulator-as-
//     operand, k order permuted to match), V^T fragments come from transposed LDS reads, and
//     the online-softmax rescale of O^T is lane-local (query on the lane);
//   * exp2 domain: t = s * scale * log2(e); p = exp2(t - m); l summed from fp32 p, P rounded
//     to bf16 for the PV product (as flash attention on the reference's GPUs).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int HD = 64;        // head dim
constexpr int WAVES = 4;
constexpr int QB = 32 * WAVES;  // query rows per workgroup
constexpr int KT = 64;        // keys per tile
constexpr int ROWB = HD * 2;  // bytes per K/V row in LDS

struct AttnArgs {
    const __hip_bfloat16* q;
    const __hip_bfloat16* k;
    const __hip_bfloat16* v;
    __hip_bfloat16* o;
    long long sqb, sqn, sqh, skb, skn, skh, svb, svn, svh, sob, son, soh;
    int N, H;
    float c;  // scale * log2(e)
};

// byte offset of 16-B chunk `ch` (0..7) of key row `key` in a [64][64 x bf16] tile image
__device__ __forceinline__ int kv_off(int key, int ch) { return key * ROWB + 16 * (ch ^ ((key >> 1) & 7)); }

// (lo, hi) -> packed bf16 pair, RNE: one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(vfm_f2{lo, hi}, vfm_bf16x2));
}

__device__ __forceinline__ float xchg32(float v) {
    // value of lane l^32 (the other half of the wave)
    return __int_as_float(__shfl_xor(__float_as_int(v), 32));
}

__global__ __launch_bounds__(64 * WAVES, 2) void attn_fwd_d64(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * KT * ROWB];  // K tile | V tile
    unsigned char* ks = lds;
    unsigned char* vs = lds + KT * ROWB;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int N = a.N;
    const int q_row = blockIdx.x * QB + 32 * wave + r;

    const __hip_bfloat16* qb = a.q + (long long)b * a.sqb + (long long)h * a.sqh;
    const __hip_bfloat16* kb = a.k + (long long)b * a.skb + (long long)h * a.skh;
    const __hip_bfloat16* vb = a.v + (long long)b * a.svb + (long long)h * a.svh;

    // Q^T B-operand fragments: lane holds Q[q_row][16s + 8hh .. +7], s = 0..3
    bf16x8 qf[4];
    {
        const bool ok = q_row < N;
        const __hip_bfloat16* qp = qb + (long long)(ok ? q_row : 0) * a.sqn + 8 * hh;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            uint4 v4 = ok ? *reinterpret_cast<const uint4*>(qp + 16 * s) : make_uint4(0, 0, 0, 0);
            qf[s] = __builtin_bit_cast(bf16x8, v4);
        }
    }

    // staging: thread t moves chunks t and t+256 of each 64 x 8-chunk tile
    const int st_key0 = tid >> 3, st_ch = tid & 7;
    uint4 kreg[2], vreg[2];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int key = t * KT + st_key0 + 32 * u;
            if (key < N) {
                kreg[u] = *reinterpret_cast<const uint4*>(kb + (long long)key * a.skn + 8 * st_ch);
                vreg[u] = *reinterpret_cast<const uint4*>(vb + (long long)key * a.svn + 8 * st_ch);
            } else {
                kreg[u] = make_uint4(0, 0, 0, 0);
                vreg[u] = make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int off = kv_off(st_key0 + 32 * u, st_ch);
            *reinterpret_cast<uint4*>(ks + off) = kreg[u];
            *reinterpret_cast<uint4*>(vs + off) = vreg[u];
        }
    };

    // transposed-read offsets of V for (key block kb, k-step s, element half e):
    // lane 4q+p of its 16-lane group reads key  32kb + 16s + 8e + 4hh + q,  d = 32db + 16g1 + 4p
    const int g1 = (lane >> 4) & 1, tq = (lane >> 2) & 3, tp = lane & 3;

    f32x16 oacc[2];
    oacc[0] = f32x16{};
    oacc[1] = f32x16{};
    float m_run = -INFINITY, l_run = 0.f;
    const float c = a.c;

    const int T = (N + KT - 1) / KT;
    load_tile(0);
    for (int t = 0; t < T; ++t) {
        store_tile();
        __syncthreads();
        if (t + 1 < T) load_tile(t + 1);

        // ---- S^T = K . Q^T for two 32-key blocks
        f32x16 sacc[2];
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            sacc[kbk] = f32x16{};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + kv_off(32 * kbk + r, 2 * s + hh));
                sacc[kbk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kbk], 0, 0, 0);
            }
        }
        // ---- mask keys beyond N (last tile only)
        const int kbase = t * KT;
        if (kbase + KT > N) {
#pragma unroll
            for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = kbase + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hh;
                    if (key >= N) sacc[kbk][i] = -INFINITY;
                }
        }
        // ---- online softmax (query = this lane's column; keys split over lane and lane^32)
        float mx = sacc[0][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mx = fmaxf(mx, sacc[0][i]);
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sacc[1][i]);
        mx = fmaxf(mx, xchg32(mx));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float ls = 0.f;
        uint32_t pk[2][8];
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[kbk][i], c, -m_new));
                const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[kbk][i + 1], c, -m_new));
                ls += p0 + p1;
                pk[kbk][i >> 1] = pack_bf16(p0, p1);
            }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            oacc[0][i] *= alpha;
            oacc[1][i] *= alpha;
        }
        // ---- O^T += V^T . P^T
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                uint4 pv;
                pv.x = pk[kbk][4 * s + 0];
                pv.y = pk[kbk][4 * s + 1];
                pv.z = pk[kbk][4 * s + 2];
                pv.w = pk[kbk][4 * s + 3];
                const bf16x8 pf = __builtin_bit_cast(bf16x8, pv);
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const int d = 32 * db + 16 * g1 + 4 * tp;
                    const int key0 = 32 * kbk + 16 * s + 4 * hh + tq;
                    const int o0 = kv_off(key0, d >> 3) + 8 * (tp & 1);
                    const int o1 = kv_off(key0 + 8, d >> 3) + 8 * (tp & 1);
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vs + o0));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vs + o1));
                    const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[db], 0, 0, 0);
                }
            }
        __syncthreads();
    }

    // ---- epilogue: O[q_row][d] = O^T[d][q_row] / l
    const float l = l_run + xchg32(l_run);
    if (q_row < N) {
        const float inv = 1.f / l;
        __hip_bfloat16* op = a.o + (long long)b * a.sob + (long long)q_row * a.son + (long long)h * a.soh;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                uint2 w;
                w.x = pack_bf16(oacc[db][4 * gi + 0] * inv, oacc[db][4 * gi + 1] * inv);
                w.y = pack_bf16(oacc[db][4 * gi + 2] * inv, oacc[db][4 * gi + 3] * inv);
                *reinterpret_cast<uint2*>(op + 32 * db + 8 * gi + 4 * hh) = w;
            }
    }
}

}  // namespace

extern "C" int vfm_attention_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int N,
                                 int head_dim, const long long* sq, const long long* sk, const long long* sv,
                                 const long long* so, float scale, void* stream) {
    if (head_dim != HD) return VFM_NO_KERNEL;
    if (!q || !k || !v || !o || !sq || !sk || !sv || !so) return VFM_ERR_ARGS;
    if (B <= 0 || H <= 0 || N <= 0 || B > 65535 || H > 65535) return VFM_ERR_ARGS;
    // 16-B vector loads of 8 bf16: every row start must be 16-B aligned (unit stride along d)
    const long long* st[4] = {sq, sk, sv, so};
    for (const long long* s : st)
        for (int i = 0; i < 3; ++i)
            if (s[i] % 8) return VFM_ERR_ARGS;
    if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16) return VFM_ERR_ARGS;
    AttnArgs a;
    a.q = (const __hip_bfloat16*)q;
    a.k = (const __hip_bfloat16*)k;
    a.v = (const __hip_bfloat16*)v;
    a.o = (__hip_bfloat16*)o;
    a.sqb = sq[0]; a.sqn = sq[1]; a.sqh = sq[2];
    a.skb = sk[0]; a.skn = sk[1]; a.skh = sk[2];
    a.svb = sv[0]; a.svn = sv[1]; a.svh = sv[2];
    a.sob = so[0]; a.son = so[1]; a.soh = so[2];
    a.N = N;
    a.H = H;
    a.c = scale * 1.4426950408889634f;
    dim3 grid((N + QB - 1) / QB, H, B);
    VFM_LAUNCH(attn_fwd_d64, grid, dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    return launch_status();
}
