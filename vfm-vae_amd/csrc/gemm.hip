// Dense GEMM on the MFMA cores with fused epilogues: the projections of the frozen ViT towers,
// the fusion adapter's projections and the decoder's 1x1 convolutions (and their backward
// products).
//
// Replaces the hipBLASLt calls behind torch.addmm / torch.bmm at
//   * HF SiglipEncoderLayer q/k/v/out_proj, fc1 (+ bias + gelu_pytorch_tanh), fc2 under bf16
//     autocast (reference networks/utils/vfms/siglip2_utils.py:121);
//   * the 1x1 convolutions / linear layers of networks/utils/convnext_utils.py:36-142
//     (modulated_pointwise_conv2d, the ConvNeXt MLP), gigagan_utils.py:53-185 (q/k/v/out, FFN)
//     and ldm_utils.py:55-166 (AttnProjection), in fp32 or bf16 as the reference runs them.
//
//   C[z] = epi( alpha * A[z] . B[z] + beta * C[z] ),   A: M x K, B: K x N, fp32 accumulation
//   epi: + bias (per column or per row), then GELU (tanh or erf form), stored bf16 or fp32.
//
// Operand layouts: each operand is "K-contiguous" (A [M][K], B [N][K] -- nn.Linear weights)
// or "MN-contiguous" (A [K][M], B [K][N] -- NCHW activations [C][HW]) with a leading
// dimension and a batch stride (0 = shared). Tiles are staged in LDS as bf16 images:
// K-contiguous operands as [128][64] (128-B rows, 16-B chunks XOR-swizzled by (row>>1)&7),
// read as MFMA fragments with ds_read_b128; MN-contiguous ones as [64][128] (256-B rows,
// the 4x4 XOR swizzle of pwgemm.hip), read with the transposing ds_read_b64_tr_b16.
//
// Precision modes (NP = bf16 pieces per operand element):
//   bf16 (NP 1): bf16 inputs, v_mfma_f32_32x32x16_bf16.
//   f32x6 (NP 3, VFM_F32, the default for fp32): fp32 inputs split on the way into LDS into
//          hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (x = hi + mid + lo exactly);
//          acc += the six piece products of order >= 2^-16 (vfm_common.h Terms<3>), each exact in
//          fp32; the dropped ones total <= ~2^-23 |a b|, one fp32 rounding: fp32-equivalent
//          products (gfx950 has no TF32/xf32; TF32 is off in the reference,
//          training_loop.py:504-505) at 2.65x the fp32 MFMA rate.
//   f32x3 (NP 2, VFM_F32X3, opt-in): hi / lo only, 3 products, <= ~2^-15.5 relative per product.
//
// Tile 128 x 128 x 64, 4 waves (2 x 2, each 64 x 64 = 2 x 2 blocks of 32 x 32), next K-tile
// prefetched into registers while the current one is multiplied (written to LDS after the
// barrier). Split-K: with `splits` > 1 each workgroup multiplies a K-range and writes fp32
// partial tiles to a workspace; vfm_gemm_reduce sums them in a fixed order (deterministic)
// and applies the epilogue.
#include "vfm_common.h"

#include <cstdlib>

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 128, BN = 128, BK = 64, THREADS = 256;
constexpr int IMG = 128 * 64 * 2;   // bytes of one bf16 tile image (either layout)

struct GemmArgs {
    const void* A;
    const void* B;
    void* C;
    const float* bias;
    float* ws;                 // split-K partials [z][splits][M][N] fp32 (null: direct epilogue)
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K, kchunk, splits;
    float alpha, beta;
    int bias_mode;             // 0 none, 1 per column (n), 2 per row (m)
    int act;                   // 0 none, 1 gelu tanh, 2 gelu erf
    // batch folding (vfm_gemm_fold): the z products of a shared A with MN-contiguous B[z] / C[z] of
    // P = 2^lgp columns each run as ONE product over N = z P columns, column n -> (batch n >> lgp,
    // column n & (P - 1)) -- per-sample planes narrower than a tile (the 8 x 8 decoder block's 1x1
    // convolutions: P = 64) fill whole tiles. 0 = off.
    int lgp;
};

// K-contiguous image [128 rows][64 k]: byte offset of 16-B chunk ch (0..7) of row
__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
// MN-contiguous image [64 k][128]: byte offset of 16-B chunk ch (0..15) of k-row
__device__ __forceinline__ int mc_off(int row, int ch) {
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}


__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    // tanh(u) = 1 - 2 / (exp(2u) + 1)
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
    return 0.5f * x * (1.f + t);
}

// ---------------------------------------------------------------------------------------
// Staging: one operand tile (128 "outer" rows x 64 k) from global memory into registers and
// from registers into its LDS image(s).
//   KCONT: global rows are outer (m or n), contiguous along k (lead = ld between rows)
//   !KCONT: global rows are k, contiguous along the outer index
// NP > 1: fp32 input split into NP bf16 images (hi, [mid,] lo), else bf16 input.
template <bool KCONT, int NP, int NT = THREADS>
struct Stage {
    static constexpr bool F32 = NP > 1;
    static constexpr int EPC = F32 ? 4 : 8;                  // elements per 16-B chunk
    static constexpr int CHUNKS = 128 * 64 / EPC;            // chunks per tile
    static constexpr int PER = CHUNKS / NT;                  // chunks per thread
    static constexpr int ROWCH = (KCONT ? 64 : 128) / EPC;   // chunks per global row of the tile
    uint4 r[PER];

    // outer0: first outer index of the tile, k0: first k, outer_n / K: bounds; lgp / sb: batch folding of
    // an MN-contiguous operand (outer index o -> batch o >> lgp at element stride sb, column o & (2^lgp - 1))
    __device__ __forceinline__ void load(const unsigned char* base, long long ld, int outer0, int k0, int outer_n,
                                         int K, int tid, int lgp = 0, long long sb = 0) {
        const int esz = F32 ? 4 : 2;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int c = tid + NT * u;
            const int row = c / ROWCH, col = (c % ROWCH) * EPC;
            int o, k;
            if (KCONT) { o = outer0 + row; k = k0 + col; }
            else       { k = k0 + row; o = outer0 + col; }
            const bool ok = (o < outer_n) && (k < K);
            long long off = KCONT ? ((long long)o * ld + k) : ((long long)k * ld + o);
            if (!KCONT && lgp) off = (long long)(o >> lgp) * sb + (long long)k * ld + (o & ((1 << lgp) - 1));
            r[u] = ok ? *reinterpret_cast<const uint4*>(base + off * esz) : make_uint4(0, 0, 0, 0);
        }
    }

    // piece p goes to img + p * IMG
    __device__ __forceinline__ void store(unsigned char* img, int tid) const {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int c = tid + NT * u;
            const int row = c / ROWCH, cc = c % ROWCH;
            if (!F32) {
                const int off = KCONT ? kc_off(row, cc) : mc_off(row, cc);
                *reinterpret_cast<uint4*>(img + off) = r[u];
            } else {
                // 4 fp32 -> 4 bf16 per piece (8 B each), half of a 16-B image chunk
                const int ch = cc >> 1, half = cc & 1;
                const int off = (KCONT ? kc_off(row, ch) : mc_off(row, ch)) + 8 * half;
                uint32_t p01[NP], p23[NP];
                split_pieces<NP>(__uint_as_float(r[u].x), __uint_as_float(r[u].y), p01);
                split_pieces<NP>(__uint_as_float(r[u].z), __uint_as_float(r[u].w), p23);
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(img + p * IMG + off) = make_uint2(p01[p], p23[p]);
            }
        }
    }
};

// MFMA operand fragment of a 32-row block `blk` (0..3 within the 128-row tile), k16 step s:
// lane (r = lane & 31, hh = lane >> 5) gets rows' k = 16s + 8hh .. +7 in natural order.
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int blk, int s, int lane) {
    const int r = lane & 31, hh = lane >> 5;
    if (KCONT) {
        return *reinterpret_cast<const bf16x8*>(img + kc_off(32 * blk + r, 2 * s + hh));
    } else {
        const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
        const int ch = 4 * blk + 2 * g1 + (p >> 1);
        const int row = 16 * s + 8 * hh + q;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row, ch) + 8 * (p & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row + 4, ch) + 8 * (p & 1)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

// NW = 4: 2 x 2 waves of 64 x 64 (one wave per SIMD for the fp32 splits: 310 registers); NW = 8: 2 x 4
// waves of 64 x 32, two waves per SIMD (<= 256 registers), so one wave's fp32 -> piece split and LDS
// stores overlap the other's MFMAs (the VGG conv's 8-wave form: 146 -> 196 TF/s there).
template <bool AK, bool BKC, int NP, bool OUTF32, int NW = 4>
__global__ __launch_bounds__(64 * NW, (NP == 3 || NW == 8) ? 1 : 2) void gemm_kernel(GemmArgs a) {
    constexpr int NT = 64 * NW, JB = NW == 8 ? 1 : 2;      // threads; 32-column blocks per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr bool F32 = NP > 1;
    unsigned char* a_img = lds;               // A pieces at a_img + p IMG
    unsigned char* b_img = lds + NP * IMG;    // B pieces at b_img + p IMG

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int tiles_n = (a.N + BN - 1) / BN;
    const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int z = blockIdx.y / a.splits, split = blockIdx.y % a.splits;
    const int kbeg = split * a.kchunk;
    const int kend = min(a.K, kbeg + a.kchunk);

    const int esz = F32 ? 4 : 2;
    const unsigned char* Ab = reinterpret_cast<const unsigned char*>(a.A) + (long long)z * a.sA * esz;
    const unsigned char* Bb = reinterpret_cast<const unsigned char*>(a.B) + (a.lgp ? 0LL : (long long)z * a.sB * esz);

    Stage<AK, NP, NT> sa;
    Stage<BKC, NP, NT> sb;
    f32x16 acc[2][JB], accs[2][JB];            // hi.hi products / the smaller piece products (NP > 1)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JB; ++j) acc[i][j] = accs[i][j] = f32x16{};

    sa.load(Ab, a.lda, m0, kbeg, a.M, kend, tid);
    sb.load(Bb, a.ldb, n0, kbeg, a.N, kend, tid, a.lgp, a.sB);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        sa.store(a_img, tid);
        sb.store(b_img, tid);
        __syncthreads();
        if (k0 + BK < kend) {
            sa.load(Ab, a.lda, m0, k0 + BK, a.M, kend, tid);
            sb.load(Bb, a.ldb, n0, k0 + BK, a.N, kend, tid, a.lgp, a.sB);
        }
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 af[NP][2], bfr[NP][JB];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
#pragma unroll
                for (int i = 0; i < 2; ++i) af[p][i] = frag<AK>(a_img + p * IMG, 2 * wm + i, s, lane);
#pragma unroll
                for (int j = 0; j < JB; ++j) bfr[p][j] = frag<BKC>(b_img + p * IMG, JB * wn + j, s, lane);
            }
            // the piece products (Terms<NP>): the smaller ones into their own accumulator (rounded
            // at their ~2^-8 scale), hi.hi alone into acc -- as many full-magnitude roundings as an
            // fp32 GEMM of exact products
#pragma unroll
            for (int t = 0; t < Terms<NP>::N; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < JB; ++j) {
                        f32x16& c = (t == Terms<NP>::N - 1) ? acc[i][j] : accs[i][j];
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[Terms<NP>::a(t)][i], bfr[Terms<NP>::b(t)][j], c,
                                                                    0, 0, 0);
                    }
        }
        __syncthreads();
    }

    if (F32) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < JB; ++j) acc[i][j] += accs[i][j];
    }

    // ---- epilogue: acc[i][j][e] = C[m][n], m = m0 + 64wm + 32i + (e&3) + 8(e>>2) + 4hh, n = n0 + 32(JB wn + j) + r
    const int r = lane & 31, hh = lane >> 5;
    if (a.ws) {   // split-K partials, raw fp32
        float* w = a.ws + ((long long)z * a.splits + split) * a.M * a.N;
#pragma unroll
        for (int j = 0; j < JB; ++j) {
            const int n = n0 + 32 * (JB * wn + j) + r;
            if (n >= a.N) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + 64 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
                    if (m < a.M) w[(long long)m * a.N + n] = acc[i][j][e];
                }
        }
        return;
    }
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* Cb = reinterpret_cast<TC*>(a.C) + (a.lgp ? 0LL : (long long)z * a.sC);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
        const int n = n0 + 32 * (JB * wn + j) + r;
        if (n >= a.N) continue;
        const float bcol = (a.bias_mode == 1) ? a.bias[a.lgp ? (n & ((1 << a.lgp) - 1)) : n] : 0.f;
        TC* Cn = a.lgp ? Cb + (long long)(n >> a.lgp) * a.sC + (n & ((1 << a.lgp) - 1)) - n : Cb;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + 64 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
                if (m >= a.M) continue;
                TC* cp = Cn + (long long)m * a.ldc + n;
                float v = a.alpha * acc[i][j][e];
                if (a.beta != 0.f) v = fmaf(a.beta, ld(cp), v);
                v += (a.bias_mode == 2) ? a.bias[m] : bcol;
                if (a.act == 1) v = gelu_tanh(v);
                else if (a.act == 2) v = v * gelu_parts(v).cdf;
                st(cp, v);
            }
    }
}

// C[z?] = epi(sum_j ws[j]) over j in [0, J): J = splits (per batch) or batches*splits (reduce_batch)
template <bool OUTF32>
__global__ void gemm_reduce_kernel(GemmArgs a, int J, int zcount) {
    const long long MN = (long long)a.M * a.N;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int z = blockIdx.y;
    if (idx >= MN) return;
    const int m = (int)(idx / a.N), n = (int)(idx % a.N);
    const float* w = a.ws + (long long)z * J * MN + idx;
    float s = 0.f;
    for (int j = 0; j < J; ++j) s += w[(long long)j * MN];
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* cp = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC + (long long)m * a.ldc + n;
    float v = a.alpha * s;
    if (a.beta != 0.f) v = fmaf(a.beta, ld(cp), v);
    v += (a.bias_mode == 2) ? a.bias[m] : (a.bias_mode == 1 ? a.bias[n] : 0.f);
    if (a.act == 1) v = gelu_tanh(v);
    else if (a.act == 2) v = v * gelu_parts(v).cdf;
    st(cp, v);
    (void)zcount;
}

template <bool AK, bool BKC, int NP, bool OUTF32, int NW>
int launch_nw(const GemmArgs& a, int batch, hipStream_t st) {
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const size_t lds = 2 * NP * IMG;
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm_kernel<AK, BKC, NP, OUTF32, NW>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr[dv_attr] = true;
    }
    VFM_LAUNCH((gemm_kernel<AK, BKC, NP, OUTF32, NW>), dim3(tiles, batch * a.splits), dim3(64 * NW), lds, st, a);
    return launch_status();
}

// waves per 128-tile workgroup for the fp32-equivalent products (8 by default; VFM_GEMM128_WAVES=4 for A/B)
int f32_waves() {
    static const int w = [] {
        const char* e = getenv("VFM_GEMM128_WAVES");
        return e && e[0] == '4' ? 4 : 8;
    }();
    return w;
}

template <bool AK, bool BKC, int NP, bool OUTF32>
int launch(const GemmArgs& a, int batch, hipStream_t st) {
    if (NP == 3 && f32_waves() == 8) return launch_nw<AK, BKC, NP, OUTF32, 8>(a, batch, st);
    return launch_nw<AK, BKC, NP, OUTF32, 4>(a, batch, st);
}

template <int NP, bool OUTF32>
int launch_layout(const GemmArgs& a, int batch, int a_kcont, int b_kcont, hipStream_t st) {
    if (a_kcont && b_kcont) return launch<true, true, NP, OUTF32>(a, batch, st);
    if (a_kcont && !b_kcont) return launch<true, false, NP, OUTF32>(a, batch, st);
    if (!a_kcont && b_kcont) return launch<false, true, NP, OUTF32>(a, batch, st);
    return launch<false, false, NP, OUTF32>(a, batch, st);
}

}  // namespace

extern "C" int vfm_gemm_workspace_floats(int M, int N, int batch, int splits, int reduce_batch) {
    (void)reduce_batch;
    if (splits <= 1 && !reduce_batch) return 0;
    return M * N * batch * (splits < 1 ? 1 : splits);
}

static int gemm_impl(const void* A, const void* B, void* C, const float* bias, float* workspace, int in_dtype,
                     int out_dtype, int M, int N, int K, int batch, int a_kcont, long long lda, long long sA,
                     int b_kcont, long long ldb, long long sB, long long ldc, long long sC, float alpha, float beta,
                     int bias_mode, int act, int splits, int reduce_batch, int lgp, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (in_dtype != VFM_BF16 && in_dtype != VFM_F32 && in_dtype != VFM_F32X3) return VFM_NO_KERNEL;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (splits < 1) splits = 1;
    // 16-B chunks along every contiguous dimension; row starts 16-B aligned
    const int epc = in_dtype == VFM_BF16 ? 8 : 4;
    const int Nrow = lgp ? (1 << lgp) : N;                      // columns of one C / B row (folded: P)
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : Nrow;
    if (a_c % epc || b_c % epc || lda % epc || ldb % epc || sA % epc || sB % epc) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    if (lgp && (b_kcont || reduce_batch || splits > 1)) return VFM_ERR_ARGS;
    if (lda < (a_kcont ? K : M) || ldb < (b_kcont ? K : Nrow) || ldc < Nrow) return VFM_ERR_ARGS;
    if ((long long)batch * splits > 65535) return VFM_ERR_ARGS;
    const bool use_ws = splits > 1 || reduce_batch;
    if (use_ws && !workspace) return VFM_ERR_ARGS;

    GemmArgs a;
    a.A = A; a.B = B; a.C = C; a.bias = bias; a.ws = use_ws ? workspace : nullptr;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K;
    a.splits = splits;
    a.kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    a.lgp = lgp;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
    int rc;
    if (in_dtype == VFM_F32) rc = of32 ? launch_layout<3, true>(a, batch, a_kcont, b_kcont, st)
                                       : launch_layout<3, false>(a, batch, a_kcont, b_kcont, st);
    else if (in_dtype == VFM_F32X3) rc = of32 ? launch_layout<2, true>(a, batch, a_kcont, b_kcont, st)
                                              : launch_layout<2, false>(a, batch, a_kcont, b_kcont, st);
    else     rc = of32 ? launch_layout<1, true>(a, batch, a_kcont, b_kcont, st)
                       : launch_layout<1, false>(a, batch, a_kcont, b_kcont, st);
    if (rc != VFM_OK || !use_ws) return rc;
    const long long MN = (long long)M * N;
    const int J = reduce_batch ? batch * splits : splits;
    const int zc = reduce_batch ? 1 : batch;
    dim3 grid((unsigned)((MN + 255) / 256), zc);
    if (of32) VFM_LAUNCH(gemm_reduce_kernel<true>, grid, dim3(256), 0, st, a, J, zc);
    else      VFM_LAUNCH(gemm_reduce_kernel<false>, grid, dim3(256), 0, st, a, J, zc);
    return launch_status();
}

extern "C" int vfm_gemm(const void* A, const void* B, void* C, const float* bias, float* workspace, int in_dtype,
                        int out_dtype, int M, int N, int K, int batch, int a_kcont, long long lda, long long sA,
                        int b_kcont, long long ldb, long long sB, long long ldc, long long sC, float alpha, float beta,
                        int bias_mode, int act, int splits, int reduce_batch, void* stream) {
    return gemm_impl(A, B, C, bias, workspace, in_dtype, out_dtype, M, N, K, batch, a_kcont, lda, sA, b_kcont, ldb, sB,
                     ldc, sC, alpha, beta, bias_mode, act, splits, reduce_batch, 0, stream);
}

// Batch-folded form: C[z] = epi(alpha A B[z] + beta C[z]) for z < batch with A shared (either layout), B[z]
// MN-contiguous [K][P] (row stride ldb, batch stride sB) and C[z] [M][P] (ldc, sC), P = 2^lgp columns
// (lgp >= 2), run as one product of N = batch * P columns. bias per row (bias_mode 2) or per column of
// the P-wide plane (1). No split-K.
extern "C" int vfm_gemm_fold(const void* A, const void* B, void* C, const float* bias, int in_dtype, int out_dtype,
                             int M, int lgp, int K, int batch, int a_kcont, long long lda, long long ldb, long long sB,
                             long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, void* stream) {
    if (lgp < 2 || lgp > 20 || batch <= 0) return VFM_ERR_ARGS;
    const long long N = (long long)batch << lgp;
    if (N > 0x7fffffffLL) return VFM_ERR_ARGS;
    const int P = 1 << lgp;
    if (ldb < P || ldc < P || sB % 8 || sC % 4) return VFM_NO_KERNEL;
    return gemm_impl(A, B, C, bias, nullptr, in_dtype, out_dtype, M, (int)N, K, 1, a_kcont, lda, 0, 0, ldb, sB, ldc, sC,
                     alpha, beta, bias_mode, act, 1, 0, lgp, stream);
}
