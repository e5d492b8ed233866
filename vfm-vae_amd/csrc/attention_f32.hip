// fp32 multi-head attention, forward + backward, on bf16 MFMA through a 3-term hi/lo split.
//
// Replaces `F.scaled_dot_product_attention(q, k, v)` on the fp32, gradient-carrying paths of
// the generator:
//   * the fusion adapter's AttnProjection (reference networks/utils/ldm_utils.py:55-87):
//     16 heads x 64, 1024 tokens (SigLIP2 @512), no autocast -> fp32;
//   * the decoder's SelfAttention with its learned null key/value (reference
//     networks/utils/gigagan_utils.py:53-91): 8 heads x 64, 1024 queries / 1025 keys, in the
//     fp32 blocks (indices 0-2 < num_fp16_res boundary).
// Both run forward and backward every G phase. AOTriton's fp32 kernels reach ~60-70 TF/s on
// these shapes; here every fp32 product a*b is evaluated as hi(a)hi(b) + hi(a)lo(b) +
// lo(a)hi(b) on v_mfma_f32_32x32x16_bf16 (hi = bf16(x), lo = bf16(x - hi); the dropped lo*lo
// term and the rounding of lo bound the relative error of each product by ~2^-16, fp32
// accumulation; gemm.hip's header has the derivation).
//
// Layout: q/k/v/o and their gradients are [B, N, H, 64] views with element strides
// (batch, token, head) and unit stride along the head dim (so the adapter's packed qkv GEMM
// output and the decoder's [B, h, P, d] tensors are read in place). lse / delta are [B, H, Nq]
// fp32, lse in the base-2 domain of the scaled scores (m + log2 l).
//
// Kernels (flash-attention-2 structure, workgroup = 4 waves x 32 rows):
//   attn32_fwd   : queries on lanes (S^T = K Q^T, swapped), online softmax, O^T = V^T P^T with
//                  the split accumulator as the B operand; writes O and lse;
//   attn32_delta : delta[q] = sum_d dO[q, d] O[q, d];
//   attn32_dq    : queries on lanes; recomputes P^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//                  dQ^T += K^T dS^T;
//   attn32_dkdv  : keys on lanes; per 64-query tile recomputes S = Q K^T, P, dP = dO V^T,
//                  dS, then dV^T += dO^T P and dK^T += Q^T dS (no atomics: dQ has its own pass).
// K/V (or Q/dO) tiles are staged fp32 -> split -> LDS as two bf16 images (128-B rows, 16-B
// chunks XOR-swizzled by (row>>1)&7, as attention.hip), next tile prefetched into registers
// during the current tile's math.
#include "vfm_common.h"

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
    float c;      // scale * log2(e)
    float scale;
};

__device__ __forceinline__ int kv_off(int row, int ch) { return row * ROWB + 16 * (ch ^ ((row >> 1) & 7)); }

// hi/lo bf16 pairs of two floats, packed
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t& h, uint32_t& l) { split2_bf16(x0, x1, h, l); }

__device__ __forceinline__ void split8(const float* x, bf16x8& h, bf16x8& l) {
    uint4 hv, lv;
    split_pair(x[0], x[1], hv.x, lv.x);
    split_pair(x[2], x[3], hv.y, lv.y);
    split_pair(x[4], x[5], hv.z, lv.z);
    split_pair(x[6], x[7], hv.w, lv.w);
    h = __builtin_bit_cast(bf16x8, hv);
    l = __builtin_bit_cast(bf16x8, lv);
}

// B-operand fragments (k step s of a 32-row accumulator block): elements 8s .. 8s+7
template <int S>
__device__ __forceinline__ void split_acc(const f32x16& a, bf16x8& h, bf16x8& l) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a[8 * S + j];
    split8(x, h, l);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// c += a * b with a = ah + al, b = bh + bl (lo * lo dropped)
__device__ __forceinline__ f32x16 mfma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
    c = mfma(al, bh, c);
    c = mfma(ah, bl, c);
    return mfma(ah, bh, c);
}

// A operand, rows of the tile image: row `row`, k = d = 16s + 8hh .. +7
__device__ __forceinline__ bf16x8 rd_row(const unsigned char* img, int row, int s, int hh) {
    return *reinterpret_cast<const bf16x8*>(img + kv_off(row, 2 * s + hh));
}

// A operand, transposed: rows = d of block db, k = tile rows of 32-row block blk, step s, in the
// k order of an accumulator block used as B operand (split_acc<s>)
struct TrLane {
    int g1, tq, tp, hh;
};
__device__ __forceinline__ bf16x8 rd_tr(const unsigned char* img, const TrLane& t, int blk, int s, int db) {
    const int d = 32 * db + 16 * t.g1 + 4 * t.tp;
    const int r0 = 32 * blk + 16 * s + 4 * t.hh + t.tq;
    const int o0 = kv_off(r0, d >> 3) + 8 * (t.tp & 1);
    const int o1 = kv_off(r0 + 8, d >> 3) + 8 * (t.tp & 1);
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
}

// register staging of one 64 x 64 fp32 tile: thread t holds row t>>2, d = 16 (t&3) .. +15
struct Stage {
    float4 v[4];
};
__device__ __forceinline__ void stage_load(Stage& s, const float* base, long long sn, int row, int nrows, int tid) {
    const int r = tid >> 2, d0 = 16 * (tid & 3);
    if (row + r < nrows) {
        const float4* p = reinterpret_cast<const float4*>(base + (long long)(row + r) * sn + d0);
#pragma unroll
        for (int u = 0; u < 4; ++u) s.v[u] = p[u];
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) s.v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
__device__ __forceinline__ void stage_store(const Stage& s, unsigned char* hi, unsigned char* lo, int tid) {
    const int r = tid >> 2, q = tid & 3;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float x[8] = {s.v[2 * c].x, s.v[2 * c].y, s.v[2 * c].z, s.v[2 * c].w,
                            s.v[2 * c + 1].x, s.v[2 * c + 1].y, s.v[2 * c + 1].z, s.v[2 * c + 1].w};
        bf16x8 h, l;
        split8(x, h, l);
        *reinterpret_cast<bf16x8*>(hi + kv_off(r, 2 * q + c)) = h;
        *reinterpret_cast<bf16x8*>(lo + kv_off(r, 2 * q + c)) = l;
    }
}

// fixed per-lane operand: row `row` of a [N, 64] fp32 matrix, d = 16s + 8hh .. +7, split
__device__ __forceinline__ void load_fixed(const float* base, long long sn, int row, int nrows, int hh, bf16x8* h,
                                           bf16x8* l) {
    const bool ok = row < nrows;
    const float* p = base + (long long)(ok ? row : 0) * sn + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        float x[8];
        if (ok) {
            const float4 a = *reinterpret_cast<const float4*>(p + 16 * s);
            const float4 b = *reinterpret_cast<const float4*>(p + 16 * s + 4);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
        }
        split8(x, h[s], l[s]);
    }
}

// store a transposed accumulator pair (rows d, lane = row of the output): out[row][d] = f * acc
__device__ __forceinline__ void store_tr(float* p, const f32x16* acc, int hh, float f) {
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int gi = 0; gi < 4; ++gi)
            *reinterpret_cast<float4*>(p + 32 * db + 8 * gi + 4 * hh) =
                make_float4(acc[db][4 * gi] * f, acc[db][4 * gi + 1] * f, acc[db][4 * gi + 2] * f, acc[db][4 * gi + 3] * f);
}

__device__ __forceinline__ float xchg32(float v) { return __int_as_float(__shfl_xor(__float_as_int(v), 32)); }

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * WAVES, 1) void attn32_fwd(Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * IMG];
    unsigned char *khi = lds, *klo = lds + IMG, *vhi = lds + 2 * IMG, *vlo = lds + 3 * IMG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk;
    const int q_row = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* kb = a.k + (long long)b * a.sk.b + (long long)h * a.sk.h;
    const float* vb = a.v + (long long)b * a.sv.b + (long long)h * a.sv.h;
    bf16x8 qh[4], ql[4];
    load_fixed(a.q + (long long)b * a.sq.b + (long long)h * a.sq.h, a.sq.n, q_row, Nq, hh, qh, ql);

    Stage sk, sv;
    f32x16 oacc[2] = {f32x16{}, f32x16{}};
    float m_run = -INFINITY, l_run = 0.f;
    const float c = a.c;
    const int T = (Nk + TT - 1) / TT;
    stage_load(sk, kb, a.sk.n, 0, Nk, tid);
    stage_load(sv, vb, a.sv.n, 0, Nk, tid);
    for (int t = 0; t < T; ++t) {
        stage_store(sk, khi, klo, tid);
        stage_store(sv, vhi, vlo, tid);
        __syncthreads();
        if (t + 1 < T) {
            stage_load(sk, kb, a.sk.n, (t + 1) * TT, Nk, tid);
            stage_load(sv, vb, a.sv.n, (t + 1) * TT, Nk, tid);
        }
        f32x16 sacc[2];
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            sacc[kbk] = f32x16{};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                sacc[kbk] = mfma3(rd_row(khi, 32 * kbk + r, s, hh), rd_row(klo, 32 * kbk + r, s, hh), qh[s], ql[s],
                                  sacc[kbk]);
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
        }
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            bf16x8 ph[2], pl[2];
            split_acc<0>(sacc[kbk], ph[0], pl[0]);
            split_acc<1>(sacc[kbk], ph[1], pl[1]);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int db = 0; db < 2; ++db)
                    oacc[db] = mfma3(rd_tr(vhi, tl, kbk, s, db), rd_tr(vlo, tl, kbk, s, db), ph[s], pl[s], oacc[db]);
        }
        __syncthreads();
    }
    const float l = l_run + xchg32(l_run);
    if (q_row < Nq) {
        store_tr(a.out + (long long)b * a.so.b + (long long)q_row * a.so.n + (long long)h * a.so.h, oacc, hh, 1.f / l);
        if (hh == 0) a.lse[((long long)b * a.H + h) * Nq + q_row] = m_run + __log2f(l);
    }
}

// ---------------------------------------------------------------------------------------------
// delta[b, h, q] = sum_d dO[b, q, h, d] * O[b, q, h, d]; one 16-lane group per row
__global__ __launch_bounds__(256) void attn32_delta(Args a, int rows) {
    const int g = (blockIdx.x * 256 + threadIdx.x) >> 4, j = threadIdx.x & 15;
    if (g >= rows) return;
    const int q = g % a.Nq, bh = g / a.Nq, h = bh % a.H, b = bh / a.H;
    const float4 o = *reinterpret_cast<const float4*>(a.o + (long long)b * a.so.b + (long long)q * a.so.n +
                                                      (long long)h * a.so.h + 4 * j);
    const float4 d = *reinterpret_cast<const float4*>(a.dout + (long long)b * a.sdo.b + (long long)q * a.sdo.n +
                                                      (long long)h * a.sdo.h + 4 * j);
    float s = o.x * d.x + o.y * d.y + o.z * d.z + o.w * d.w;
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (j == 0) a.delta[g] = s;
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * WAVES, 2) void attn32_dq(Args a) {   // 2 waves per SIMD (the register budget the kernel was tuned to)
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * IMG];
    unsigned char *khi = lds, *klo = lds + IMG, *vhi = lds + 2 * IMG, *vlo = lds + 3 * IMG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk;
    const int q_row = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* kb = a.k + (long long)b * a.sk.b + (long long)h * a.sk.h;
    const float* vb = a.v + (long long)b * a.sv.b + (long long)h * a.sv.h;
    bf16x8 qh[4], ql[4], oh[4], ol[4];
    load_fixed(a.q + (long long)b * a.sq.b + (long long)h * a.sq.h, a.sq.n, q_row, Nq, hh, qh, ql);
    load_fixed(a.dout + (long long)b * a.sdo.b + (long long)h * a.sdo.h, a.sdo.n, q_row, Nq, hh, oh, ol);
    const long long rix = ((long long)b * a.H + h) * Nq + (q_row < Nq ? q_row : 0);
    const float lse = q_row < Nq ? a.lse[rix] : INFINITY;
    const float dlt = q_row < Nq ? a.delta[rix] : 0.f;

    Stage sk, sv;
    f32x16 dq[2] = {f32x16{}, f32x16{}};
    const float c = a.c;
    const int T = (Nk + TT - 1) / TT;
    stage_load(sk, kb, a.sk.n, 0, Nk, tid);
    stage_load(sv, vb, a.sv.n, 0, Nk, tid);
    for (int t = 0; t < T; ++t) {
        stage_store(sk, khi, klo, tid);
        stage_store(sv, vhi, vlo, tid);
        __syncthreads();
        if (t + 1 < T) {
            stage_load(sk, kb, a.sk.n, (t + 1) * TT, Nk, tid);
            stage_load(sv, vb, a.sv.n, (t + 1) * TT, Nk, tid);
        }
        const int kbase = t * TT;
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk) {
            f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                s = mfma3(rd_row(khi, 32 * kbk + r, st, hh), rd_row(klo, 32 * kbk + r, st, hh), qh[st], ql[st], s);
                dp = mfma3(rd_row(vhi, 32 * kbk + r, st, hh), rd_row(vlo, 32 * kbk + r, st, hh), oh[st], ol[st], dp);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = kbase + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const float p = key < Nk ? __builtin_amdgcn_exp2f(fmaf(s[i], c, -lse)) : 0.f;
                s[i] = p * (dp[i] - dlt);
            }
            bf16x8 dh[2], dl[2];
            split_acc<0>(s, dh[0], dl[0]);
            split_acc<1>(s, dh[1], dl[1]);
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int db = 0; db < 2; ++db)
                    dq[db] = mfma3(rd_tr(khi, tl, kbk, st, db), rd_tr(klo, tl, kbk, st, db), dh[st], dl[st], dq[db]);
        }
        __syncthreads();
    }
    if (q_row < Nq)
        store_tr(a.dq + (long long)b * a.sdq.b + (long long)q_row * a.sdq.n + (long long)h * a.sdq.h, dq, hh, a.scale);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * WAVES, 1) void attn32_dkdv(Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * IMG + 2 * TT * 4];
    unsigned char *qhi = lds, *qlo = lds + IMG, *ohi = lds + 2 * IMG, *olo = lds + 3 * IMG;
    float* lse_s = reinterpret_cast<float*>(lds + 4 * IMG);
    float* dlt_s = lse_s + TT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int h = blockIdx.y, b = blockIdx.z;
    const int Nq = a.Nq, Nk = a.Nk;
    const int key = blockIdx.x * RB + 32 * wave + r;
    const TrLane tl{(lane >> 4) & 1, (lane >> 2) & 3, lane & 3, hh};

    const float* qb = a.q + (long long)b * a.sq.b + (long long)h * a.sq.h;
    const float* ob = a.dout + (long long)b * a.sdo.b + (long long)h * a.sdo.h;
    const float* lb = a.lse + ((long long)b * a.H + h) * Nq;
    const float* db_ = a.delta + ((long long)b * a.H + h) * Nq;
    bf16x8 kh[4], kl[4], vh[4], vl[4];
    load_fixed(a.k + (long long)b * a.sk.b + (long long)h * a.sk.h, a.sk.n, key, Nk, hh, kh, kl);
    load_fixed(a.v + (long long)b * a.sv.b + (long long)h * a.sv.h, a.sv.n, key, Nk, hh, vh, vl);

    Stage sq, so;
    float lse_r = INFINITY, dlt_r = 0.f;
    auto load_rows = [&](int q0) {
        stage_load(sq, qb, a.sq.n, q0, Nq, tid);
        stage_load(so, ob, a.sdo.n, q0, Nq, tid);
        if (tid < TT) {
            const bool ok = q0 + tid < Nq;
            lse_r = ok ? lb[q0 + tid] : INFINITY;
            dlt_r = ok ? db_[q0 + tid] : 0.f;
        }
    };
    f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
    const float c = a.c;
    const int T = (Nq + TT - 1) / TT;
    load_rows(0);
    for (int t = 0; t < T; ++t) {
        stage_store(sq, qhi, qlo, tid);
        stage_store(so, ohi, olo, tid);
        if (tid < TT) {
            lse_s[tid] = lse_r;
            dlt_s[tid] = dlt_r;
        }
        __syncthreads();
        if (t + 1 < T) load_rows((t + 1) * TT);
#pragma unroll
        for (int qbk = 0; qbk < 2; ++qbk) {
            f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                s = mfma3(rd_row(qhi, 32 * qbk + r, st, hh), rd_row(qlo, 32 * qbk + r, st, hh), kh[st], kl[st], s);
                dp = mfma3(rd_row(ohi, 32 * qbk + r, st, hh), rd_row(olo, 32 * qbk + r, st, hh), vh[st], vl[st], dp);
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
            bf16x8 ph[2], pl[2], dh[2], dl[2];
            split_acc<0>(s, ph[0], pl[0]);
            split_acc<1>(s, ph[1], pl[1]);
            split_acc<0>(dp, dh[0], dl[0]);
            split_acc<1>(dp, dh[1], dl[1]);
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int d = 0; d < 2; ++d) {
                    dv[d] = mfma3(rd_tr(ohi, tl, qbk, st, d), rd_tr(olo, tl, qbk, st, d), ph[st], pl[st], dv[d]);
                    dk[d] = mfma3(rd_tr(qhi, tl, qbk, st, d), rd_tr(qlo, tl, qbk, st, d), dh[st], dl[st], dk[d]);
                }
        }
        __syncthreads();
    }
    if (key < Nk) {
        store_tr(a.dk + (long long)b * a.sdk.b + (long long)key * a.sdk.n + (long long)h * a.sdk.h, dk, hh, a.scale);
        store_tr(a.dv + (long long)b * a.sdv.b + (long long)key * a.sdv.n + (long long)h * a.sdv.h, dv, hh, 1.f);
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

int check_shape(int B, int H, int Nq, int Nk, int head_dim) {
    if (head_dim != HD) return VFM_NO_KERNEL;
    if (B <= 0 || H <= 0 || Nq <= 0 || Nk <= 0 || B > 65535 || H > 65535) return VFM_ERR_ARGS;
    return VFM_OK;
}

}  // namespace

extern "C" int vfm_attention_f32_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int H,
                                     int Nq, int Nk, int head_dim, const long long* sq, const long long* sk,
                                     const long long* sv, const long long* so, float scale, void* stream) {
    int rc = check_shape(B, H, Nq, Nk, head_dim);
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
    hipLaunchKernelGGL(attn32_fwd, dim3((Nq + RB - 1) / RB, H, B), dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    return launch_status();
}

extern "C" int vfm_attention_f32_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                     const void* lse, void* delta, void* dq, void* dk, void* dv, int B, int H, int Nq,
                                     int Nk, int head_dim, const long long* sq, const long long* sk,
                                     const long long* sv, const long long* so, const long long* sdo,
                                     const long long* sdq, const long long* sdk, const long long* sdv, float scale,
                                     void* stream) {
    int rc = check_shape(B, H, Nq, Nk, head_dim);
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
    hipStream_t st = (hipStream_t)stream;
    const long long rows = (long long)B * H * Nq;
    if (rows > (1ll << 31) / 16) return VFM_ERR_ARGS;
    hipLaunchKernelGGL(attn32_delta, dim3((unsigned)((rows * 16 + 255) / 256)), dim3(256), 0, st, a, (int)rows);
    hipLaunchKernelGGL(attn32_dq, dim3((Nq + RB - 1) / RB, H, B), dim3(64 * WAVES), 0, st, a);
    hipLaunchKernelGGL(attn32_dkdv, dim3((Nk + RB - 1) / RB, H, B), dim3(64 * WAVES), 0, st, a);
    return launch_status();
}
