// Large-tile bf16 GEMM for the hot path's big products (the frozen ViT projections, the fusion
// adapter and the decoder's 1x1 convolutions at batch 32): C[z] = epi(alpha A[z] B[z] + beta C[z]).
// Same contract and epilogue as csrc/gemm.hip (vfm_gemm); this is the path vfm_gemm takes when
// K is a multiple of 64 and the operands are bf16 (fp32 operands arrive here pre-split as
// [hi | hi | lo] x [hi ; lo ; hi] along K, see vfm_split3 below: the 3-term product as ONE
// bf16 GEMM of depth 3K).
//
// Structure (cdna_hip_programming.md §5: "The 256² template", "glds vs register staging"):
//   * workgroup tile 256 x 256 x 64, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 =
//     8 x 4 blocks of v_mfma_f32_16x16x32_bf16 (32 accumulators, 128 VGPRs);
//   * operand tiles move HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane,
//     no register staging), two stages of 64 KB, the next K-tile's DMA issued before the
//     current tile's MFMAs and retired with a counted `s_waitcnt vmcnt(8)`, raw s_barrier
//     (no __syncthreads: its fence would drain the in-flight DMA);
//   * LDS images are XOR-swizzled on the SOURCE address (the DMA destination is lane-linear):
//     K-contiguous operands [256][64] with 128-B rows, chunk ^= (row>>1)&7, read as MFMA
//     fragments with ds_read_b128 (conflict-free); MN-contiguous operands [64][256] with
//     512-B rows, chunk ^= 2*((row&3) | ((row>>3)&1)<<2), read with ds_read_b64_tr_b16;
//   * workgroup -> tile mapping is XCD-aware: the 8 blocks b, b+8, ... that share an XCD's L2
//     take consecutive tiles of one tile row (they share the A panel).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int FBM = 256, FBN = 256, FBK = 64, FTHREADS = 512;
constexpr int FIMG = 256 * 64 * 2;           // bytes of one operand image (32 KB)
constexpr int FSTAGE = 2 * FIMG;             // A + B

struct FastArgs {
    const __hip_bfloat16* A;
    const __hip_bfloat16* B;
    void* C;
    const float* bias;
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K;
    float alpha, beta;
    int bias_mode, act;
};

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mc_swz(int row) { return 2 * ((row & 3) | (((row >> 3) & 1) << 2)); }
__device__ __forceinline__ int mc_off(int row, int ch) { return row * 512 + 16 * (ch ^ mc_swz(row)); }

__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f));
}

// Issue the LDS-DMA of one operand tile (rows r0.. of a K-contiguous operand, or k-rows k0.. of
// an MN-contiguous one) into `img`; 4 x 16 B per thread.
template <bool KCONT>
__device__ __forceinline__ void dma_tile(unsigned char* img, const __hip_bfloat16* base, long long ld, int outer0,
                                         int outer_n, int k0, int tid) {
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int cbase = wave * 64 + 512 * u;           // wave-uniform first chunk of this instruction
        const int ci = cbase + lane;
        const __hip_bfloat16* src;
        if (KCONT) {
            const int row = ci >> 3, chs = (ci & 7) ^ ((row >> 1) & 7);
            const int o = min(outer0 + row, outer_n - 1);
            src = base + (long long)o * ld + k0 + 8 * chs;
        } else {
            const int row = ci >> 5, chs = (ci & 31) ^ mc_swz(row);
            int o = outer0 + 8 * chs;
            if (o >= outer_n) o = 0;                       // (outer_n % 8 == 0): a valid chunk, result unused
            src = base + (long long)(k0 + row) * ld + o;
        }
        __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + cbase * 16), 16, 0, 0);
    }
}

// 16x16x32 operand fragment of 16-row block `blk`, k32 step t: lane l holds rows' k = 32t + 8(l>>4) + j.
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag16(const unsigned char* img, int blk, int t, int lane) {
    if (KCONT) {
        return *reinterpret_cast<const bf16x8*>(img + kc_off(16 * blk + (lane & 15), 4 * t + (lane >> 4)));
    } else {
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int ch = 2 * blk + (p >> 1);
        const int row = 32 * t + 8 * g + q;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row, ch) + 8 * (p & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row + 4, ch) + 8 * (p & 1)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

template <bool AK, bool BKC, bool OUTF32>
__global__ __launch_bounds__(FTHREADS, 1) void gemm_fast_kernel(FastArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int tiles_m = (a.M + FBM - 1) / FBM, tiles_n = (a.N + FBN - 1) / FBN;
    const int nwg = tiles_m * tiles_n;
    // XCD-aware bijective remap (blocks b, b+8, ... share an XCD): consecutive tiles per XCD
    const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const int m0 = tm * FBM, n0 = tn * FBN;
    const int z = blockIdx.y;
    const __hip_bfloat16* Ab = a.A + (long long)z * a.sA;
    const __hip_bfloat16* Bb = a.B + (long long)z * a.sB;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

    const int KT = a.K / FBK;
    dma_tile<AK>(lds, Ab, a.lda, m0, a.M, 0, tid);
    dma_tile<BKC>(lds + FIMG, Bb, a.ldb, n0, a.N, 0, tid);
    for (int kt = 0; kt < KT; ++kt) {
        unsigned char* cur = lds + (kt & 1) * FSTAGE;
        if (kt + 1 < KT) {
            unsigned char* nxt = lds + ((kt + 1) & 1) * FSTAGE;
            dma_tile<AK>(nxt, Ab, a.lda, m0, a.M, (kt + 1) * FBK, tid);
            dma_tile<BKC>(nxt + FIMG, Bb, a.ldb, n0, a.N, (kt + 1) * FBK, tid);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            // all fragments of this k32 step first (12 reads in flight), then 32 MFMAs
            bf16x8 bf[4], af[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = frag16<BKC>(cur + FIMG, 4 * wn + j, t, lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) af[i] = frag16<AK>(cur, 8 * wm + i, t, lane);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

    // epilogue: acc[i][j][r] = C[m0 + 128wm + 16i + 4(l>>4) + r][n0 + 64wn + 16j + (l&15)]
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* Cb = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC;
    const int cl = lane & 15, rq = 4 * (lane >> 4);
    if (!OUTF32 && a.beta == 0.f && m0 + FBM <= a.M && n0 + FBN <= a.N && (a.ldc % 8) == 0 &&
        (reinterpret_cast<uintptr_t>(a.C) % 16) == 0 && (a.sC % 8) == 0) {
        // bf16 tile through LDS (the main loop's 128 KB are free after the last barrier): each
        // wave writes its 128 x 64 block as bf16 rows of 128 B, then stores whole 16-B chunks
        unsigned short* wl = reinterpret_cast<unsigned short*>(lds + wave * 128 * 128);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int nl = 16 * j + cl;
            const int n = n0 + 64 * wn + nl;
            const float bcol = (a.bias_mode == 1) ? a.bias[n] : 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ml = 16 * i + rq + r;
                    float v = a.alpha * acc[i][j][r];
                    v += (a.bias_mode == 2) ? a.bias[m0 + 128 * wm + ml] : bcol;
                    if (a.act == 1) v = gelu_tanh(v);
                    else if (a.act == 2) v = v * gelu_parts(v).cdf;
                    // row ml, 16-B chunk (nl>>3) XOR-swizzled by row to spread the 2-byte writes
                    const int ch = (nl >> 3) ^ (ml & 7);
                    wl[ml * 64 + ch * 8 + (nl & 7)] = __builtin_bit_cast(unsigned short, __float2bfloat16(v));
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        __hip_bfloat16* crow = reinterpret_cast<__hip_bfloat16*>(a.C) + (long long)z * a.sC +
                               (long long)(m0 + 128 * wm) * a.ldc + n0 + 64 * wn;
#pragma unroll 4
        for (int c = lane; c < 128 * 8; c += 64) {
            const int ml = c >> 3, chl = c & 7;
            const uint4 v = *reinterpret_cast<const uint4*>(wl + ml * 64 + 8 * (chl ^ (ml & 7)));
            *reinterpret_cast<uint4*>(crow + (long long)ml * a.ldc + 8 * chl) = v;
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + 64 * wn + 16 * j + cl;
        if (n >= a.N) continue;
        const float bcol = (a.bias_mode == 1) ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 128 * wm + 16 * i + rq + r;
                if (m >= a.M) continue;
                TC* cp = Cb + (long long)m * a.ldc + n;
                float v = a.alpha * acc[i][j][r];
                if (a.beta != 0.f) v = fmaf(a.beta, ld(cp), v);
                v += (a.bias_mode == 2) ? a.bias[m] : bcol;
                if (a.act == 1) v = gelu_tanh(v);
                else if (a.act == 2) v = v * gelu_parts(v).cdf;
                st(cp, v);
            }
    }
}

template <bool AK, bool BKC, bool OUTF32>
int launch_fast(const FastArgs& a, int batch, hipStream_t st) {
    const int nwg = ((a.M + FBM - 1) / FBM) * ((a.N + FBN - 1) / FBN);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gemm_fast_kernel<AK, BKC, OUTF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * FSTAGE);
        attr = true;
    }
    hipLaunchKernelGGL((gemm_fast_kernel<AK, BKC, OUTF32>), dim3(nwg, batch), dim3(FTHREADS), 2 * FSTAGE, st, a);
    return launch_status();
}

// fp32 -> bf16 3-term split along the reduction dimension (see the file header).
//   role 0 (A operand): parts (hi, hi, lo); role 1 (B operand): parts (hi, lo, hi).
//   kcont = 1: src [R][K] (row stride lds), dst [R][3K]; kcont = 0: src [K][R], dst [3K][R].
__global__ void split3_kernel(const float* __restrict__ src, __hip_bfloat16* __restrict__ dst, int R, int K,
                              long long lds_, long long sb, long long db, int role, int kcont) {
    const long long idx4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const long long total = (long long)R * K;
    if (idx4 >= total) return;
    const int z = blockIdx.y;
    const float* s = src + (long long)z * sb;
    __hip_bfloat16* d = dst + (long long)z * db;
    // 4 consecutive elements along the contiguous dimension
    long long r, c, inner;
    if (kcont) { r = idx4 / K; c = idx4 % K; inner = K; }
    else       { r = idx4 / R; c = idx4 % R; inner = R; }   // r = k row, c = column
    const float4 v = *reinterpret_cast<const float4*>(s + r * lds_ + c);
    uint32_t h01, l01, h23, l23;
    split2_bf16(v.x, v.y, h01, l01);
    split2_bf16(v.z, v.w, h23, l23);
    const uint2 H = make_uint2(h01, h23);
    const uint2 L = make_uint2(l01, l23);
    const uint2 parts[3] = {H, role == 0 ? H : L, role == 0 ? L : H};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        long long off;
        if (kcont) off = r * (3LL * K) + (long long)p * K + c;
        else       off = ((long long)p * K + r) * inner + c;
        *reinterpret_cast<uint2*>(d + off) = parts[p];
    }
}

}  // namespace

extern "C" int vfm_gemm_fast(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N,
                             int K, int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb,
                             long long sB, long long ldc, long long sC, float alpha, float beta, int bias_mode, int act,
                             void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (K % FBK) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    if (lda < (a_kcont ? K : M) || ldb < (b_kcont ? K : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + FBM - 1) / FBM) * ((N + FBN - 1) / FBN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    FastArgs a;
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
#define VFM_FAST(AK, BK_)                                                                     \
    return of32 ? launch_fast<AK, BK_, true>(a, batch, st) : launch_fast<AK, BK_, false>(a, batch, st)
    if (a_kcont && b_kcont) VFM_FAST(true, true);
    if (a_kcont && !b_kcont) VFM_FAST(true, false);
    if (!a_kcont && b_kcont) VFM_FAST(false, true);
    VFM_FAST(false, false);
#undef VFM_FAST
}

extern "C" int vfm_split3(const float* src, void* dst, int R, int K, long long ld, long long sb, long long db, int batch,
                          int role, int kcont, void* stream) {
    if (!src || !dst || R <= 0 || K <= 0 || batch <= 0 || batch > 65535 || (role != 0 && role != 1)) return VFM_ERR_ARGS;
    const int inner = kcont ? K : R;
    if (inner % 4 || ld % 4 || sb % 4 || ((uintptr_t)src % 16) || ((uintptr_t)dst % 8)) return VFM_NO_KERNEL;
    const long long total4 = ((long long)R * K) / 4;
    dim3 grid((unsigned)((total4 + 255) / 256), batch);
    hipLaunchKernelGGL(split3_kernel, grid, dim3(256), 0, (hipStream_t)stream, src, (__hip_bfloat16*)dst, R, K, ld,
                       sb, db, role, kcont);
    return launch_status();
}
