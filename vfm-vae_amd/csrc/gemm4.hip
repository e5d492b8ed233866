// 256 x 256 bf16 GEMM with one wave per SIMD: the frozen SigLIP2 tower's linears and the decoder's bf16
// 1x1 convolutions (C[z] = epi(alpha A[z] B[z] + beta C[z])).
//
// Why a second 256-tile kernel beside gemm8: gemm8 runs 8 waves (two per SIMD, 128 x 64 each, 256
// registers) in a ping-pong of 8 barriers per K-tile. Here the 4 waves of a workgroup each own a
// 128 x 128 block (8 x 8 v_mfma_f32_16x16x32_bf16 tiles), so a wave has the SIMD's whole 512-entry
// register file: 256 accumulator registers, a register stage of the next K-tile (64), the fragments
// of one k32 step (64), and one barrier per K-tile. Per K-tile a wave issues 128 MFMAs (2048 SIMD
// cycles) beside 32 fragment reads, 16 global loads and 16 LDS writes.
//
//   * operand tiles [256][64] (K-contiguous) or [64][256] (M/N-contiguous) go global -> registers
//     (buffer loads, one VGPR offset per chunk, the K-tile advance a scalar offset) -> LDS (two
//     64 KB stages); the K-tile t+2 loads are issued while K-tile t computes, their LDS write
//     during K-tile t+1;
//   * LDS images: K-contiguous [256 rows][64 k] with 128-B rows, chunk ^= (row >> 1) & 7
//     (ds_read_b128 fragments); MN-contiguous as two [64 k][128] halves, 256-B rows, the 4 x 4
//     chunk swizzle of the transposed reads (ds_read_b64_tr_b16) -- the images of gemm8.hip;
//   * the MFMA takes the B fragment as its first operand, so the accumulator of a 16 x 16 tile
//     holds, per lane, 4 CONSECUTIVE columns of one C row: the epilogue stores straight from the
//     accumulators (8-B bf16 / 16-B fp32 per lane), no LDS staging;
//   * XCD-aware bijective block -> tile remap with grouped tile order (as gemm8).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64, THREADS = 256;
constexpr int OPB = 256 * BK * 2;          // bytes of one operand tile image (32 KB)
constexpr int STAGE = 2 * OPB;             // A + B images of one K-tile (64 KB)

struct G4Args {
    const __hip_bfloat16* A;
    const __hip_bfloat16* B;
    void* C;
    const float* bias;
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K;
    float alpha, beta;
    int bias_mode, act, out_f32;
    unsigned spanA, spanB;   // buffer-descriptor ranges in bytes (< 2^31, checked on the host)
};

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mc_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int mc_off(int row, int ch) { return row * 256 + 16 * (ch ^ mc_swz(row)); }

__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f));
}

// 16x16x32 operand fragment of 16-row (or 16-column) block `blk` of an operand image, k32 step t:
// lane l carries row (col) l & 15, k = 32 t + 8 (l >> 4) .. + 7.
//   K-contiguous image [256][64]: blk 0..15;
//   MN-contiguous image: two [64][128] halves of 16 KB, blk 0..15 (half blk >> 3).
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int blk, int t, int lane) {
    if (KCONT) {
        return *reinterpret_cast<const bf16x8*>(img + kc_off(16 * blk + (lane & 15), 4 * t + (lane >> 4)));
    } else {
        const unsigned char* h = img + (blk >> 3) * (OPB / 2);
        const int b = blk & 7;
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int ch = 2 * b + (p >> 1);
        const int row = 32 * t + 8 * g + q;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(h + mc_off(row, ch) + 8 * (p & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(h + mc_off(row + 4, ch) + 8 * (p & 1)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

// Per-thread chunk i (0..7) of an operand tile: global byte offset relative to the K-tile origin and
// the LDS byte offset inside the operand image. K-contiguous: row (tid >> 3) + 32 i, 16-B chunk tid & 7
// (rows beyond outer_n clamped: their results are never stored). MN-contiguous: k-row (tid >> 5) + 8 i,
// chunk tid & 31 of the 256 columns (columns beyond outer_n read chunk 0: outer_n % 8 == 0).
template <bool KCONT>
__device__ __forceinline__ void chunk_offsets(long long ld, int outer0, int outer_n, int i, int tid, unsigned& gofs,
                                              int& lofs) {
    if (KCONT) {
        const int row = (tid >> 3) + 32 * i, ch = tid & 7;
        const int o = min(outer0 + row, outer_n - 1);
        gofs = (unsigned)(((long long)o * ld + 8 * ch) * 2);
        lofs = kc_off(row, ch);
    } else {
        const int krow = (tid >> 5) + 8 * i, ch = tid & 31;
        int o = outer0 + 8 * ch;
        if (o >= outer_n) o = 0;
        gofs = (unsigned)(((long long)krow * ld + o) * 2);
        lofs = (ch >> 4) * (OPB / 2) + mc_off(krow, ch & 15);
    }
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    const f2 x = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, b2));
}

// alpha, beta C, bias and activation of 4 consecutive columns n.. of row m (rolled: the epilogue's
// 64 tiles stay small code)
__device__ __forceinline__ f32x4 epi4(const G4Args& a, f32x4 v, const void* rowp, int m, int n) {
    const float brow = (a.bias_mode == 2 && m < a.M) ? a.bias[m] : 0.f;
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
        const bool in = n + r < a.N && m < a.M;
        float x = a.alpha * v[r];
        if (a.beta != 0.f && in) {
            const float c = a.out_f32 ? reinterpret_cast<const float*>(rowp)[n + r]
                                      : ld(reinterpret_cast<const __hip_bfloat16*>(rowp) + n + r);
            x = fmaf(a.beta, c, x);
        }
        x += (a.bias_mode == 1) ? (in ? a.bias[n + r] : 0.f) : brow;
        if (a.act == 1) x = gelu_tanh(x);
        else if (a.act == 2) x = x * gelu_parts(x).cdf;
        v[r] = x;
    }
    return v;
}

template <bool OUTF32, class TC>
__device__ __forceinline__ void store4(TC* row, int n, f32x4 v, bool mok, bool whole, int N) {
    if (!mok) return;
    if (whole) {
        if (OUTF32) *reinterpret_cast<f32x4*>(row + n) = v;
        else *reinterpret_cast<uint2*>(row + n) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    } else {
        for (int r = 0; r < 4; ++r)
            if (n + r < N) st(row + n + r, v[r]);
    }
}

template <bool AK, bool BKC, bool OUTF32>
__global__ __launch_bounds__(THREADS, 1) void gemm4_kernel(G4Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    int m0, n0;
    {
        const int bid = blockIdx.x;
        const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        constexpr int GROUP = 4;
        const int gsz = GROUP * tiles_n, grp = tile / gsz, rem = tile - grp * gsz;
        const int rows_g = min(GROUP, tiles_m - grp * GROUP);
        m0 = (grp * GROUP + rem % rows_g) * BM;
        n0 = (rem / rows_g) * BN;
    }
    const int z = blockIdx.y;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)a.spanA, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)a.spanB, 0x00020000);
    unsigned gA[8], gB[8];
    int lA[8], lB[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        chunk_offsets<AK>(a.lda, m0, a.M, i, tid, gA[i], lA[i]);
        chunk_offsets<BKC>(a.ldb, n0, a.N, i, tid, gB[i], lB[i]);
    }
    const long long zA = (long long)z * a.sA * 2, zB = (long long)z * a.sB * 2;
    const int KT = a.K / BK;
    uint4 stg[16];
    auto gload = [&](int kt) {
        const unsigned sa = (unsigned)(zA + (AK ? (long long)kt * BK * 2 : (long long)kt * BK * a.lda * 2));
        const unsigned sb = (unsigned)(zB + (BKC ? (long long)kt * BK * 2 : (long long)kt * BK * a.ldb * 2));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            stg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rA, gA[i], sa, 0));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            stg[8 + i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rB, gB[i], sb, 0));
    };
    auto swrite = [&](int buf) {
        unsigned char* base = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(base + lA[i]) = stg[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(base + OPB + lB[i]) = stg[8 + i];
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};

    gload(0);
    swrite(0);
    if (KT > 1) gload(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // A blocks of this wave: rows 128 wm + 16 bi -> image block 8 wm + bi (both layouts); same for B
    const int ablk = 8 * wm, bblk = 8 * wn;
    for (int kt = 0; kt < KT; ++kt) {
        const unsigned char* buf = lds + (kt & 1) * STAGE;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            bf16x8 af[8], bf[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) af[i] = frag<AK>(buf, ablk + i, t, lane);
#pragma unroll
            for (int j = 0; j < 8; ++j) bf[j] = frag<BKC>(buf + OPB, bblk + j, t, lane);
            if (t == 1 && kt + 1 < KT) {
                swrite((kt + 1) & 1);
                if (kt + 2 < KT) gload(kt + 2);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

    // epilogue: acc[i][j][r] = C[m0 + 128 wm + 16 i + (lane & 15)][n0 + 128 wn + 16 j + 4 (lane >> 4) + r]
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* Cz = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC;
    const bool plain = a.beta == 0.f && a.bias_mode == 0 && a.act == 0 && a.alpha == 1.f;
    const bool vec = (a.ldc % 4) == 0 && (a.sC % 4) == 0 && (reinterpret_cast<uintptr_t>(a.C) % 16) == 0;
    const int mb = m0 + 128 * wm + (lane & 15), nb = n0 + 128 * wn + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = mb + 16 * i;
        const bool mok = m < a.M;
        TC* row = Cz + (long long)min(m, a.M - 1) * a.ldc;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = nb + 16 * j;
            f32x4 v = acc[i][j];
            if (!plain) v = epi4(a, v, row, m, n);
            store4<OUTF32>(row, n, v, mok, vec && n + 4 <= a.N, a.N);
        }
    }
}

template <bool AK, bool BKC, bool OUTF32>
void launch4(const G4Args& a, int batch, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gemm4_kernel<AK, BKC, OUTF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * STAGE);
        attr = true;
    }
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    VFM_LAUNCH((gemm4_kernel<AK, BKC, OUTF32>), dim3(nwg, batch), dim3(THREADS), 2 * STAGE, st, a);
}

long long span4(int kcont, long long outer, long long kdim, long long ld, long long sb, int batch) {
    const long long rows = kcont ? outer : kdim;
    const long long cols = kcont ? kdim : outer;
    const long long e = (rows - 1) * ld + cols + (long long)(batch - 1) * sb;
    const long long bytes = e * 2;
    return bytes >= (1LL << 31) ? -1 : bytes;
}

}  // namespace

// bf16 operands: C[z] (M x N, ldc, batch stride sC) = epi(alpha A[z] B[z] + beta C[z]) with A [M, K]
// (a_kcont: K-contiguous rows of stride lda, else M-contiguous rows of K) and B [K, N] (b_kcont: B is
// given as N rows of K, stride ldb; else K rows of N). bias_mode 0 none / 1 per column / 2 per row;
// act 0 none / 1 tanh-GELU / 2 erf-GELU. Returns VFM_NO_KERNEL for shapes it does not take (K % 64,
// unaligned operands, > 2 GiB spans).
extern "C" int vfm_gemm4(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N, int K,
                         int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                         long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (K % BK) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    if (lda < (a_kcont ? (long long)K : M) || ldb < (b_kcont ? (long long)K : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    const long long spA = span4(a_kcont, M, K, lda, sA, batch);
    const long long spB = span4(b_kcont, N, K, ldb, sB, batch);
    if (spA < 0 || spB < 0) return VFM_NO_KERNEL;
    G4Args a{};
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    a.spanA = (unsigned)spA; a.spanB = (unsigned)spB;
    a.out_f32 = out_dtype == VFM_F32;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
#define VFM_G4(AK, BK_) of32 ? launch4<AK, BK_, true>(a, batch, st) : launch4<AK, BK_, false>(a, batch, st)
    if (a_kcont && b_kcont) VFM_G4(true, true);
    else if (a_kcont && !b_kcont) VFM_G4(true, false);
    else if (!a_kcont && b_kcont) VFM_G4(false, true);
    else VFM_G4(false, false);
#undef VFM_G4
    return launch_status();
}
