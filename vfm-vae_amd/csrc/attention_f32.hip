// fp32 multi-head attention, forward + backward, on bf16 MFMA with fp32-equivalent products (the
// f32x6 split of vfm_common.h: three exact bf16 pieces per operand, six piece products; the 3-term
// f32x3 split is an opt-in precision code).
//
// Replaces `F.scaled_dot_product_attention(q, k, v)` on the fp32, gradient-carrying paths of
// the generator:
//   * the fusion adapter's AttnProjection (reference networks/utils/ldm_utils.py:55-87):
//     16 heads x 64, 1024 tokens (SigLIP2 @512), no autocast -> fp32;
//   * the decoder's SelfAttention with its learned null key/value (reference
//     networks/utils/gigagan_utils.py:53-91): 8 heads x 64, 1024 queries / 1025 keys, in the
//     fp32 blocks (indices 0-2 < num_fp16_res boundary).
//   * the decode-side AttnProjection (post_quant, ldm_utils.py:480-488): 16 heads x 32;
//   * the DINO ViT-S discriminator tower (6 heads x 64, 197 tokens).
// Both generator paths run forward and backward every G phase. Every fp32 product a*b is evaluated
// as the Terms<NP> piece products on v_mfma_f32_32x32x16_bf16 (NP = 3: hi, mid, lo with
// x = hi + mid + lo exactly; the dropped products total <= ~2^-23 |a b|), fp32 accumulation.
//
// Layout: q/k/v/o and their gradients are [B, N, H, d] views (d = 64, or 32: staged into the same
// 64-wide images with zeros in d >= 32, so the products are unchanged and only d < 32 is stored)
// with element strides (batch, token, head) and unit stride along the head dim (so the adapter's
// packed qkv GEMM output and the decoder's [B, h, P, d] tensors are read in place). lse / delta are
// [B, H, Nq] fp32, lse in the base-2 domain of the scaled scores (m + log2 l).
//
// Kernels (flash-attention-2 structure, workgroup = 4 waves x 32 rows):
//   attn32_fwd   : queries on lanes (S^T = K Q^T, swapped), online softmax, O^T = V^T P^T with
//                  the split accumulator as the B operand; writes O and lse;
//   attn32_delta : delta[q] = sum_d dO[q, d] O[q, d];
//   attn32_dq    : queries on lanes; recomputes P^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//                  dQ^T += K^T dS^T;
//   attn32_dkdv  : keys on lanes; per 64-query tile recomputes S = Q K^T, P, dP = dO V^T,
//                  dS, then dV^T += dO^T P and dK^T += Q^T dS (no atomics: dQ has its own pass).
// K/V (or Q/dO) tiles are staged fp32 -> split -> LDS as NP bf16 images (128-B rows, 16-B chunks
// XOR-swizzled by (row>>1)&7, as attention.hip), next tile prefetched into registers during the
// current tile's math.
#include "vfm_common.h"

#include <cstdlib>

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int HD = 64;
constexpr int WAVES = 4;
constexpr int RB = 32 * WAVES;   // rows (queries or keys) owned by a workgroup
constexpr int TT = 64;           // rows per streamed tile
constexpr int ROWB = HD * 2;     // bytes per bf16 row image
constexpr int IMG = TT * ROWB;   // bytes per tile image

struct Strides {
    long long b, n, h;
};

struct Args {
    const float *q, *k, *v, *o, *dout;
    float *out, *lse, *delta, *dq, *dk, *dv;
    Strides sq, sk, sv, so, sdo, sdq, sdk, sdv;
    int Nq, Nk, H;
    int hd;       // head dim of the tensors: 64, or 32 (zero-extended to 64 on chip)
    float c;      // scale * log2(e)
    float scale;
};

__device__ __forceinline__ int kv_off(int row, int ch) { return row * ROWB + 16 * (ch ^ ((row >> 1) & 7)); }

// one operand fragment as its NP bf16 pieces
template <int NP>
struct Frag {
    bf16x8 p[NP];
};

// 8 floats -> NP bf16x8 pieces
template <int NP>
__device__ __forceinline__ Frag<NP> split8(const float* x) {
    uint32_t q[4][NP];
#pragma unroll
    for (int j = 0; j < 4; ++j) split_pieces<NP>(x[2 * j], x[2 * j + 1], q[j]);
    Frag<NP> f;
#pragma unroll
    for (int p = 0; p < NP; ++p) f.p[p] = __builtin_bit_cast(bf16x8, make_uint4(q[0][p], q[1][p], q[2][p], q[3][p]));
    return f;
}

// B-operand fragments (k step s of a 32-row accumulator block): elements 8s .. 8s+7
template <int NP, int S>
__device__ __forceinline__ Frag<NP> split_acc(const f32x16& a) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a[8 * S + j];
    return split8<NP>(x);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// c += a * b over the piece products (Terms<NP>, smallest first)
template <int NP>
__device__ __forceinline__ f32x16 mfmaN(const Frag<NP>& a, const Frag<NP>& b, f32x16 c) {
#pragma unroll
    for (int t = 0; t < Terms<NP>::N; ++t) c = mfma(a.p[Terms<NP>::a(t)], b.p[Terms<NP>::b(t)], c);
    return c;
}

// the same with the smaller piece products into their own accumulator cs and hi.hi alone into c
// (for the long reductions over keys / queries: full-magnitude roundings as in an fp32 GEMM of
// exact products; cs is added once at the end)
template <int NP>
__device__ __forceinline__ void mfmaN2(const Frag<NP>& a, const Frag<NP>& b, f32x16& c, f32x16& cs) {
#pragma unroll
    for (int t = 0; t < Terms<NP>::N - 1; ++t) cs = mfma(a.p[Terms<NP>::a(t)], b.p[Terms<NP>::b(t)], cs);
    c = mfma(a.p[0], b.p[0], c);
}

// A operand, rows of the tile images (piece p at img + p IMG): row `row`, k = d = 16s + 8hh .. +7
template <int NP>
__device__ __forceinline__ Frag<NP> rd_row(const unsigned char* img, int row, int s, int hh) {
    Frag<NP> f;
#pragma unroll
    for (int p = 0; p < NP; ++p) f.p[p] = *reinterpret_cast<const bf16x8*>(img + p * IMG + kv_off(row, 2 * s + hh));
    return f;
}

// A operand, transposed: rows = d of block db, k = tile rows of 32-row block blk, step s, in the
// k order of an accumulator block used as B operand (split_acc<s>)
struct TrLane {
    int g1, tq, tp, hh;
};
template <int NP>
__device__ __forceinline__ Frag<NP> rd_tr(const unsigned char* img, const TrLane& t, int blk, int s, int db) {
    const int d = 32 * db + 16 * t.g1 + 4 * t.tp;
    const int r0 = 32 * blk + 16 * s + 4 * t.hh + t.tq;
    const int o0 = kv_off(r0, d >> 3) + 8 * (t.tp & 1);
    const int o1 = kv_off(r0 + 8, d >> 3) + 8 * (t.tp & 1);
    Frag<NP> f;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + p * IMG + o0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + p * IMG + o1));
        f.p[p] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
    }
    return f;
}

// register staging of one 64 x 64 fp32 tile: thread t holds row t>>2, d = 16 (t&3) .. +15
// (zeros for d >= hd)
struct Stage {
    float4 v[4];
};
__device__ __forceinline__ void stage_load(Stage& s, const float* base, long long sn, int row, int nrows, int hd,
                                           int tid) {
    const int r = tid >> 2, d0 = 16 * (tid & 3);
    if (row + r < nrows && d0 < hd) {
        const float4* p = reinterpret_cast<const float4*>(base + (long long)(row + r) * sn + d0);
#pragma unroll
        for (int u = 0; u < 4; ++u) s.v[u] = p[u];
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) s.v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
template <int NP>
__device__ __forceinline__ void stage_store(const Stage& s, unsigned char* img, int tid) {
    const int r = tid >> 2, q = tid & 3;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float x[8] = {s.v[2 * c].x, s.v[2 * c].y, s.v[2 * c].z, s.v[2 * c].w,
                            s.v[2 * c + 1].x, s.v[2 * c + 1].y, s.v[2 * c + 1].z, s.v[2 * c + 1].w};
        const Frag<NP> f = split8<NP>(x);
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<bf16x8*>(img + p * IMG + kv_off(r, 2 * q + c)) = f.p[p];
    }
}

// fixed per-lane operand: row `row` of a [N, hd] fp32 matrix, d = 16s + 8hh .. +7 (zero for
// d >= hd), split into pieces
template <int NP>
__device__ __forceinline__ void load_fixed(const float* base, long long sn, int row, int nrows, int hd, int hh,
                                           Frag<NP>* f) {
    const bool ok = row < nrows;
    const float* p = base + (long long)(ok ? row : 0) * sn + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        float x[8];
        if (ok && 16 * s < hd) {
            const float4 a = *reinterpret_cast<const float4*>(p + 16 * s);
            const float4 b = *reinterpret_cast<const float4*>(p + 16 * s + 4);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
        }
        f[s] = split8<NP>(x);
    }
}

// store a transposed accumulator pair (rows d, lane = row of the output): out[row][d] = f * acc, d < hd
__device__ __forceinline__ void store_tr(float* p, const f32x16* acc, int hh, float f, int hd) {
#pragma unroll
    for (int db = 0; db < 2; ++db)
        if (32 * db < hd)
#pragma unroll
        for (int gi = 0; gi < 4; ++gi)
            *reinterpret_cast<float4*>(p + 32 * db + 8 * gi + 4 * hh) =
                make_float4(acc[db][4 * gi] * f, acc[db][4 * gi + 1] * f, acc[db][4 * gi + 2] * f, acc[db][4 * gi + 3] * f);
}

__device__ __forceinline__ float xchg32(float v) { return __int_as_float(__shfl_xor(__float_as_int(v), 32)); }

// ---------------------------------------------------------------------------------------------
// OCC = 1: the next K/V tile prefetched into registers during the current tile's math (one wave per
// SIMD: 292 registers); OCC = 2 (default): no register prefetch, 220 registers and two workgroups per
// CU, so one workgroup's softmax / piece splits / loads overlap the other's MFMAs (PMC: 6.6 VALU
// instructions per 32x32x16 MFMA; MI355X: adapter shape 1110 -> 965 us, decoder 32 x 32 489 -> 398 us,
// DINO 38 -> 29.5 us, profiles/r4_o_attn32_occ.txt). VFM_ATTN32_OCC=1 selects the prefetch form.
template <int NP, int OCC>
__global__ __launch_bounds__(64 * WAVES, OCC) void attn32_fwd(Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * NP * IMG];
    unsigned char *kimg = lds, *vimg = lds + NP * IMG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk, hd = a.hd;
    const int q_row = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* kb = a.k + (long long)b * a.sk.b + (long long)h * a.sk.h;
    const float* vb = a.v + (long long)b * a.sv.b + (long long)h * a.sv.h;
    Frag<NP> qf[4];
    load_fixed<NP>(a.q + (long long)b * a.sq.b + (long long)h * a.sq.h, a.sq.n, q_row, Nq, hd, hh, qf);

    Stage sk, sv;
    f32x16 oacc[2] = {f32x16{}, f32x16{}}, oaccs[2] = {f32x16{}, f32x16{}};
    float m_run = -INFINITY, l_run = 0.f;
    const float c = a.c;
    const int T = (Nk + TT - 1) / TT;
    if (OCC == 1) {
        stage_load(sk, kb, a.sk.n, 0, Nk, hd, tid);
        stage_load(sv, vb, a.sv.n, 0, Nk, hd, tid);
    }
    for (int t = 0; t < T; ++t) {
        if (OCC != 1) {
            stage_load(sk, kb, a.sk.n, t * TT, Nk, hd, tid);
            stage_load(sv, vb, a.sv.n, t * TT, Nk, hd, tid);
        }
        stage_store<NP>(sk, kimg, tid);
        stage_store<NP>(sv, vimg, tid);
        __syncthreads();
        if (OCC == 1 && t + 1 < T) {
            stage_load(sk, kb, a.sk.n, (t + 1) * TT, Nk, hd, tid);
            stage_load(sv, vb, a.sv.n, (t + 1) * TT, Nk, hd, tid);
        }
        f32x16 sacc[2];
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            sacc[kbk] = f32x16{};
#pragma unroll
            for (int s = 0; s < 4; ++s) sacc[kbk] = mfmaN<NP>(rd_row<NP>(kimg, 32 * kbk + r, s, hh), qf[s], sacc[kbk]);
        }
        const int kbase = t * TT;
        if (kbase + TT > Nk) {
#pragma unroll
            for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (kbase + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hh >= Nk) sacc[kbk][i] = -INFINITY;
        }
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
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kbk][i], c, -m_new));
                sacc[kbk][i] = p;
                ls += p;
            }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            oacc[0][i] *= alpha;
            oacc[1][i] *= alpha;
            oaccs[0][i] *= alpha;
            oaccs[1][i] *= alpha;
        }
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            const Frag<NP> pf[2] = {split_acc<NP, 0>(sacc[kbk]), split_acc<NP, 1>(sacc[kbk])};
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int db = 0; db < 2; ++db) mfmaN2<NP>(rd_tr<NP>(vimg, tl, kbk, s, db), pf[s], oacc[db], oaccs[db]);
        }
        __syncthreads();
    }
    oacc[0] += oaccs[0];
    oacc[1] += oaccs[1];
    const float l = l_run + xchg32(l_run);
    if (q_row < Nq) {
        store_tr(a.out + (long long)b * a.so.b + (long long)q_row * a.so.n + (long long)h * a.so.h, oacc, hh, 1.f / l,
                 hd);
        if (hh == 0) a.lse[((long long)b * a.H + h) * Nq + q_row] = m_run + __log2f(l);
    }
}

// ---------------------------------------------------------------------------------------------
// delta[b, h, q] = sum_d dO[b, q, h, d] * O[b, q, h, d]; one 16-lane group per row (4 floats a lane)
__global__ __launch_bounds__(256) void attn32_delta(Args a, int rows) {
    const int g = (blockIdx.x * 256 + threadIdx.x) >> 4, j = threadIdx.x & 15;
    if (g >= rows) return;
    const int q = g % a.Nq, bh = g / a.Nq, h = bh % a.H, b = bh / a.H;
    float s = 0.f;
    if (4 * j < a.hd) {
        const float4 o = *reinterpret_cast<const float4*>(a.o + (long long)b * a.so.b + (long long)q * a.so.n +
                                                          (long long)h * a.so.h + 4 * j);
        const float4 d = *reinterpret_cast<const float4*>(a.dout + (long long)b * a.sdo.b + (long long)q * a.sdo.n +
                                                          (long long)h * a.sdo.h + 4 * j);
        s = o.x * d.x + o.y * d.y + o.z * d.z + o.w * d.w;
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (j == 0) a.delta[g] = s;
}

// ---------------------------------------------------------------------------------------------
// OCC as in attn32_fwd: OCC = 1 prefetches the next K/V tile into registers (one wave per SIMD for
// NP = 3), OCC = 2 loads it after the barrier and fits two workgroups per CU.
template <int NP, int OCC>
__global__ __launch_bounds__(64 * WAVES, OCC) void attn32_dq(Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * NP * IMG];
    unsigned char *kimg = lds, *vimg = lds + NP * IMG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk, hd = a.hd;
    const int q_row = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* kb = a.k + (long long)b * a.sk.b + (long long)h * a.sk.h;
    const float* vb = a.v + (long long)b * a.sv.b + (long long)h * a.sv.h;
    Frag<NP> qf[4], of[4];
    load_fixed<NP>(a.q + (long long)b * a.sq.b + (long long)h * a.sq.h, a.sq.n, q_row, Nq, hd, hh, qf);
    load_fixed<NP>(a.dout + (long long)b * a.sdo.b + (long long)h * a.sdo.h, a.sdo.n, q_row, Nq, hd, hh, of);
    const long long rix = ((long long)b * a.H + h) * Nq + (q_row < Nq ? q_row : 0);
    const float lse = q_row < Nq ? a.lse[rix] : INFINITY;
    const float dlt = q_row < Nq ? a.delta[rix] : 0.f;

    Stage sk, sv;
    f32x16 dq[2] = {f32x16{}, f32x16{}}, dqs[2] = {f32x16{}, f32x16{}};
    const float c = a.c;
    const int T = (Nk + TT - 1) / TT;
    if (OCC == 1) {
        stage_load(sk, kb, a.sk.n, 0, Nk, hd, tid);
        stage_load(sv, vb, a.sv.n, 0, Nk, hd, tid);
    }
    for (int t = 0; t < T; ++t) {
        if (OCC != 1) {
            stage_load(sk, kb, a.sk.n, t * TT, Nk, hd, tid);
            stage_load(sv, vb, a.sv.n, t * TT, Nk, hd, tid);
        }
        stage_store<NP>(sk, kimg, tid);
        stage_store<NP>(sv, vimg, tid);
        __syncthreads();
        if (OCC == 1 && t + 1 < T) {
            stage_load(sk, kb, a.sk.n, (t + 1) * TT, Nk, hd, tid);
            stage_load(sv, vb, a.sv.n, (t + 1) * TT, Nk, hd, tid);
        }
        const int kbase = t * TT;
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                s = mfmaN<NP>(rd_row<NP>(kimg, 32 * kbk + r, st, hh), qf[st], s);
                dp = mfmaN<NP>(rd_row<NP>(vimg, 32 * kbk + r, st, hh), of[st], dp);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = kbase + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const float p = key < Nk ? __builtin_amdgcn_exp2f(fmaf(s[i], c, -lse)) : 0.f;
                s[i] = p * (dp[i] - dlt);
            }
            const Frag<NP> df[2] = {split_acc<NP, 0>(s), split_acc<NP, 1>(s)};
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int db = 0; db < 2; ++db) mfmaN2<NP>(rd_tr<NP>(kimg, tl, kbk, st, db), df[st], dq[db], dqs[db]);
        }
        __syncthreads();
    }
    dq[0] += dqs[0];
    dq[1] += dqs[1];
    if (q_row < Nq)
        store_tr(a.dq + (long long)b * a.sdq.b + (long long)q_row * a.sdq.n + (long long)h * a.sdq.h, dq, hh, a.scale,
                 hd);
}

// ---------------------------------------------------------------------------------------------
// OCC = 1 (VFM_ATTN32_DKDV_OCC=1): Q / dO tile prefetch in registers, the small piece products of dK /
// dV in accumulators of their own (420 registers, one wave per SIMD). OCC = 2 (default): no prefetch,
// one accumulator per output block (all six piece products summed into it, as the S / dP products
// are) and P's / dS's pieces live one after the other -- 248 registers, two workgroups per CU:
// attention backward -11 % on the adapter / decoder shapes, within the same error bounds (2x torch's
// exact fp32 error, tests/test_attention_f32_gpu.py), profiles/r4_ah_attn32_dkdv_occ.txt.
template <int NP, int OCC>
__global__ __launch_bounds__(64 * WAVES, OCC) void attn32_dkdv(Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * NP * IMG + 2 * TT * 4];
    unsigned char *qimg = lds, *oimg = lds + NP * IMG;
    float* lse_s = reinterpret_cast<float*>(lds + 2 * NP * IMG);
    float* dlt_s = lse_s + TT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk, hd = a.hd;
    const int key = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* qb = a.q + (long long)b * a.sq.b + (long long)h * a.sq.h;
    const float* ob = a.dout + (long long)b * a.sdo.b + (long long)h * a.sdo.h;
    const float* lb = a.lse + ((long long)b * a.H + h) * Nq;
    const float* db_ = a.delta + ((long long)b * a.H + h) * Nq;
    Frag<NP> kf[4], vf[4];
    load_fixed<NP>(a.k + (long long)b * a.sk.b + (long long)h * a.sk.h, a.sk.n, key, Nk, hd, hh, kf);
    load_fixed<NP>(a.v + (long long)b * a.sv.b + (long long)h * a.sv.h, a.sv.n, key, Nk, hd, hh, vf);

    Stage sq, so;
    float lse_r = INFINITY, dlt_r = 0.f;
    auto load_rows = [&](int q0) {
        stage_load(sq, qb, a.sq.n, q0, Nq, hd, tid);
        stage_load(so, ob, a.sdo.n, q0, Nq, hd, tid);
        if (tid < TT) {
            const bool ok = q0 + tid < Nq;
            lse_r = ok ? lb[q0 + tid] : INFINITY;
            dlt_r = ok ? db_[q0 + tid] : 0.f;
        }
    };
    f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
    f32x16 dks[2] = {f32x16{}, f32x16{}}, dvs[2] = {f32x16{}, f32x16{}};
    const float c = a.c;
    const int T = (Nq + TT - 1) / TT;
    if (OCC == 1) load_rows(0);
    for (int t = 0; t < T; ++t) {
        if (OCC != 1) load_rows(t * TT);
        stage_store<NP>(sq, qimg, tid);
        stage_store<NP>(so, oimg, tid);
        if (tid < TT) {
            lse_s[tid] = lse_r;
            dlt_s[tid] = dlt_r;
        }
        __syncthreads();
        if (OCC == 1 && t + 1 < T) load_rows((t + 1) * TT);
#pragma unroll
        for (int qbk = 0; qbk < 2; ++qbk) {
            f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                s = mfmaN<NP>(rd_row<NP>(qimg, 32 * qbk + r, st, hh), kf[st], s);
                dp = mfmaN<NP>(rd_row<NP>(oimg, 32 * qbk + r, st, hh), vf[st], dp);
            }
            // rows of this lane's accumulator entries: 32 qbk + 8 gi + 4 hh + (0..3)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                const float4 L = *reinterpret_cast<const float4*>(lse_s + 32 * qbk + 8 * gi + 4 * hh);
                const float4 D = *reinterpret_cast<const float4*>(dlt_s + 32 * qbk + 8 * gi + 4 * hh);
                const float Ls[4] = {L.x, L.y, L.z, L.w}, Ds[4] = {D.x, D.y, D.z, D.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int i = 4 * gi + j;
                    const float p = __builtin_amdgcn_exp2f(fmaf(s[i], c, -Ls[j]));
                    s[i] = p;
                    dp[i] = p * (dp[i] - Ds[j]);
                }
            }
            if (OCC == 1) {
                const Frag<NP> pf[2] = {split_acc<NP, 0>(s), split_acc<NP, 1>(s)};
                const Frag<NP> df[2] = {split_acc<NP, 0>(dp), split_acc<NP, 1>(dp)};
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int d = 0; d < 2; ++d) {
                        mfmaN2<NP>(rd_tr<NP>(oimg, tl, qbk, st, d), pf[st], dv[d], dvs[d]);
                        mfmaN2<NP>(rd_tr<NP>(qimg, tl, qbk, st, d), df[st], dk[d], dks[d]);
                    }
            } else {
                {
                    const Frag<NP> pf[2] = {split_acc<NP, 0>(s), split_acc<NP, 1>(s)};
#pragma unroll
                    for (int st = 0; st < 2; ++st)
#pragma unroll
                        for (int d = 0; d < 2; ++d) dv[d] = mfmaN<NP>(rd_tr<NP>(oimg, tl, qbk, st, d), pf[st], dv[d]);
                }
                const Frag<NP> df[2] = {split_acc<NP, 0>(dp), split_acc<NP, 1>(dp)};
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int d = 0; d < 2; ++d) dk[d] = mfmaN<NP>(rd_tr<NP>(qimg, tl, qbk, st, d), df[st], dk[d]);
            }
        }
        __syncthreads();
    }
    if (OCC == 1) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            dk[d] += dks[d];
            dv[d] += dvs[d];
        }
    }
    if (key < Nk) {
        store_tr(a.dk + (long long)b * a.sdk.b + (long long)key * a.sdk.n + (long long)h * a.sdk.h, dk, hh, a.scale, hd);
        store_tr(a.dv + (long long)b * a.sdv.b + (long long)key * a.sdv.n + (long long)h * a.sdv.h, dv, hh, 1.f, hd);
    }
}

bool strides_ok(const long long* s) {
    if (!s) return false;
    for (int i = 0; i < 3; ++i)
        if (s[i] % 4) return false;   // 16-B float4 rows
    return true;
}
Strides mk(const long long* s) { return Strides{s[0], s[1], s[2]}; }
bool aligned16(const void* p) { return ((uintptr_t)p % 16) == 0; }

int check_shape(int B, int H, int Nq, int Nk, int head_dim, int precision) {
    if (head_dim != HD && head_dim != 32) return VFM_NO_KERNEL;
    if (precision != VFM_F32 && precision != VFM_F32X3) return VFM_ERR_ARGS;
    if (B <= 0 || H <= 0 || Nq <= 0 || Nk <= 0 || B > 65535 || H > 65535) return VFM_ERR_ARGS;
    return VFM_OK;
}

}  // namespace

extern "C" int vfm_attention_f32_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int H,
                                     int Nq, int Nk, int head_dim, const long long* sq, const long long* sk,
                                     const long long* sv, const long long* so, float scale, int precision,
                                     void* stream) {
    int rc = check_shape(B, H, Nq, Nk, head_dim, precision);
    if (rc != VFM_OK) return rc;
    if (!q || !k || !v || !o || !lse) return VFM_ERR_ARGS;
    if (!strides_ok(sq) || !strides_ok(sk) || !strides_ok(sv) || !strides_ok(so)) return VFM_ERR_ARGS;
    if (!aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o)) return VFM_ERR_ARGS;
    Args a{};
    a.q = (const float*)q; a.k = (const float*)k; a.v = (const float*)v;
    a.out = (float*)o; a.lse = (float*)lse;
    a.sq = mk(sq); a.sk = mk(sk); a.sv = mk(sv); a.so = mk(so);
    a.Nq = Nq; a.Nk = Nk; a.H = H;
    a.scale = scale;
    a.c = scale * 1.4426950408889634f;
    a.hd = head_dim;
    const dim3 grid((Nq + RB - 1) / RB, H, B);
    static const int occ = [] {
        const char* e = getenv("VFM_ATTN32_OCC");
        return e && e[0] == '1' ? 1 : 2;
    }();
    if (precision == VFM_F32) {
        if (occ == 2) VFM_LAUNCH((attn32_fwd<3, 2>), grid, dim3(64 * WAVES), 0, (hipStream_t)stream, a);
        else VFM_LAUNCH((attn32_fwd<3, 1>), grid, dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    } else {
        VFM_LAUNCH((attn32_fwd<2, 1>), grid, dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    }
    return launch_status();
}

extern "C" int vfm_attention_f32_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                     const void* lse, void* delta, void* dq, void* dk, void* dv, int B, int H, int Nq,
                                     int Nk, int head_dim, const long long* sq, const long long* sk,
                                     const long long* sv, const long long* so, const long long* sdo,
                                     const long long* sdq, const long long* sdk, const long long* sdv, float scale,
                                     int precision, void* stream) {
    int rc = check_shape(B, H, Nq, Nk, head_dim, precision);
    if (rc != VFM_OK) return rc;
    if (!q || !k || !v || !o || !dout || !lse || !delta || !dq || !dk || !dv) return VFM_ERR_ARGS;
    const long long* ss[8] = {sq, sk, sv, so, sdo, sdq, sdk, sdv};
    for (const long long* s : ss)
        if (!strides_ok(s)) return VFM_ERR_ARGS;
    const void* ps[8] = {q, k, v, o, dout, dq, dk, dv};
    for (const void* p : ps)
        if (!aligned16(p)) return VFM_ERR_ARGS;
    Args a{};
    a.q = (const float*)q; a.k = (const float*)k; a.v = (const float*)v; a.o = (const float*)o;
    a.dout = (const float*)dout; a.lse = (float*)lse; a.delta = (float*)delta;
    a.dq = (float*)dq; a.dk = (float*)dk; a.dv = (float*)dv;
    a.sq = mk(sq); a.sk = mk(sk); a.sv = mk(sv); a.so = mk(so); a.sdo = mk(sdo);
    a.sdq = mk(sdq); a.sdk = mk(sdk); a.sdv = mk(sdv);
    a.Nq = Nq; a.Nk = Nk; a.H = H;
    a.scale = scale;
    a.c = scale * 1.4426950408889634f;
    a.hd = head_dim;
    hipStream_t st = (hipStream_t)stream;
    const long long rows = (long long)B * H * Nq;
    if (rows > (1ll << 31) / 16) return VFM_ERR_ARGS;
    VFM_LAUNCH(attn32_delta, dim3((unsigned)((rows * 16 + 255) / 256)), dim3(256), 0, st, a, (int)rows);
    const dim3 gq((Nq + RB - 1) / RB, H, B), gk((Nk + RB - 1) / RB, H, B);
    static const int dq_occ = [] {
        const char* e = getenv("VFM_ATTN32_DQ_OCC");
        return e && e[0] == '1' ? 1 : 2;
    }();
    static const int dkdv_occ = [] {
        const char* e = getenv("VFM_ATTN32_DKDV_OCC");
        return e && e[0] == '1' ? 1 : 2;
    }();
    if (precision == VFM_F32) {
        if (dq_occ == 2) VFM_LAUNCH((attn32_dq<3, 2>), gq, dim3(64 * WAVES), 0, st, a);
        else VFM_LAUNCH((attn32_dq<3, 1>), gq, dim3(64 * WAVES), 0, st, a);
        if (dkdv_occ == 2) VFM_LAUNCH((attn32_dkdv<3, 2>), gk, dim3(64 * WAVES), 0, st, a);
        else VFM_LAUNCH((attn32_dkdv<3, 1>), gk, dim3(64 * WAVES), 0, st, a);
    } else {
        VFM_LAUNCH((attn32_dq<2, 2>), gq, dim3(64 * WAVES), 0, st, a);
        VFM_LAUNCH((attn32_dkdv<2, 1>), gk, dim3(64 * WAVES), 0, st, a);
    }
    return launch_status();
}
