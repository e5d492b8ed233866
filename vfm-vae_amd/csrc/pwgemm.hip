// The ConvNeXt MLP's channel GEMM with its GELU fused into the epilogue (bf16, MFMA).
//
// Reference: ConvNeXtSynthesisLayer (convnext_utils.py:121-142) computes, per sample b,
//   h = W1 . m_b   (modulated 1x1 conv C -> 4C, here a shared-weight GEMM; the per-(b,o)
//                   demodulation is the epilogue scale s[b,o])
//   g = GELU(h * s[b,o] + bias[o])
// and in backward dh = (W2^T . dy) * GELU'(h*s+b) * s, d_s[b,o] = sum_p dz*h, d_bias = sum dz.
// Unfused, the 4C-channel tensors h and dg each make an extra HBM round trip through a
// separate elementwise kernel; with K = C in {128, 256, 512} these GEMMs are HBM-bound
// (4C x P outputs against a C x P input), so the round trips are most of their cost.
//
//   mode 0 (forward):  out0 = bf16(acc)            (h, only when backward will need it)
//                      out1 = bf16(GELU(bf16(acc) * s + bias))
//   mode 1 (backward): dg = bf16(acc); z = h*s + bias; dz = dg * GELU'(z)
//                      out0 = bf16(dz * s); part0[b, tile, m] = sum_n dz*h; part1 = sum_n dz
// bf16(acc) is rounded before the epilogue uses it, as the unfused path rounds the GEMM's
// bf16 output, so both paths see the same operand.
//
// Layout: A [M, K] row-major (W1, or W2^T), X [B, K, N] (channels x pixels), outputs
// [B, M, N]. One workgroup = one sample x 128 pixel columns; it stages X[b][:, n0:n0+128]
// once in LDS (K rows of 256 B, 16-B chunks XOR-swizzled) and sweeps all M rows in steps
// of 128 (4 waves x 32 rows), so X is read from HBM exactly once. A fragments come straight
// from global memory (the weight is tiny and L2-resident). v_mfma_f32_32x32x16_bf16:
// A lane l holds A[r][8h+j] (r = l&31, h = l>>5), B lane l holds B[8h+j][r], taken from the
// row-major X image with two ds_read_b64_tr_b16; C/D: col = l&31, row = (i&3)+8(i>>2)+4h.
//
// Status: parity-tested (tests/test_pwgemm_gpu.py), not yet on the training path. Measured
// at batch 32 (tools_dev/pwbench.py, MI355X): forward with h written 1.33 ms vs 1.67 ms for
// bmm + GELU kernel at C=128 / 256^2, 0.82 vs 0.90 ms at C=256 / 128^2, but 0.87 vs 0.61 ms
// at C=512 / 64^2; backward 2-4x slower than the unfused pair. The epilogue is VALU-bound
// (GELU math on 4C x P elements with 2 waves/SIMD), not store-bound: staging the tile through
// LDS for whole-row stores was slower. Next: packed-f32 epilogue math, more waves per SIMD.
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int NT = 128;   // pixel columns per workgroup
constexpr int WAVES = 4;  // each wave owns 32 output rows of every 128-row M step

struct PwArgs {
    const __hip_bfloat16* A;
    const __hip_bfloat16* X;
    const float* scale;        // [B, M] or null
    const float* bias;         // [M] or null
    const __hip_bfloat16* h;   // mode 1: [B, M, N]
    __hip_bfloat16* out0;
    __hip_bfloat16* out1;
    float* part0;
    float* part1;
    int M, N, ntiles;
};

// byte offset of 16-B chunk `ch` (0..15) of row `row` in a [rows][128 x bf16] image
__device__ __forceinline__ int swz(int row, int ch) {
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ float bf16_round(float v) { return __bfloat162float(__float2bfloat16(v)); }

template <int MODE, int K>
__global__ __launch_bounds__(256) void pw_gemm_gelu(PwArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y;
    const int tile = blockIdx.x;
    const int n0 = tile * NT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int M = a.M, N = a.N;

    const __hip_bfloat16* xb = a.X + (long long)b * K * N + n0;
#pragma unroll 4
    for (int i = tid; i < K * 16; i += 256) {
        const int row = i >> 4, ch = i & 15;
        const uint4 v = *reinterpret_cast<const uint4*>(xb + (long long)row * N + ch * 8);
        *reinterpret_cast<uint4*>(lds + swz(row, ch)) = v;
    }
    __syncthreads();

    const int r = lane & 31, hh = lane >> 5;
    const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    // transposed-read byte offsets for k-step 0; rows advance by 16 per k-step (the XOR term
    // depends on row & 15 only, so the offset of k-step s is base + 16 * 256 * s)
    int tro[4][2];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
        const int c0 = 4 * nb + 2 * g1 + (p >> 1);
        tro[nb][0] = swz(8 * hh + q, c0) + 8 * (p & 1);
        tro[nb][1] = swz(8 * hh + 4 + q, c0) + 8 * (p & 1);
    }

    const long long outb = (long long)b * M * N + n0 + r;
    for (int mc = 0; mc < M; mc += 32 * WAVES) {
        const int m0 = mc + 32 * wave;
        const __hip_bfloat16* arow = a.A + (long long)(m0 + r) * K + 8 * hh;
        f32x16 acc[4];
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x16{};
        bf16x8 af[K / 16];
#pragma unroll
        for (int s = 0; s < K / 16; ++s) af[s] = *reinterpret_cast<const bf16x8*>(arow + 16 * s);
#pragma unroll
        for (int s = 0; s < K / 16; ++s) {
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(lds + tro[nb][0] + 4096 * s));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(lds + tro[nb][1] + 4096 * s));
                const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], __builtin_bit_cast(bf16x8, both),
                                                                  acc[nb], 0, 0, 0);
            }
        }

        // epilogue: register i of acc[nb] is row m0 + (i&3) + 8(i>>2) + 4hh, column n0 + 32nb + r
        if (MODE == 0) {
            // direct per-lane stores: staging the tile through LDS for whole-row stores measured
            // slower (the epilogue is VALU-bound, not store-bound)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const float sc = a.scale ? a.scale[(long long)b * M + m] : 1.f;
                const float bi = a.bias ? a.bias[m] : 0.f;
                const long long row = outb + (long long)m * N;
#pragma unroll
                for (int nb = 0; nb < 4; ++nb) {
                    const __hip_bfloat16 hv = __float2bfloat16(acc[nb][i]);
                    if (a.out0) a.out0[row + 32 * nb] = hv;
                    const float z = fmaf(__bfloat162float(hv), sc, bi);
                    a.out1[row + 32 * nb] = __float2bfloat16(z * gelu_parts(z).cdf);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const float sc = a.scale ? a.scale[(long long)b * M + m] : 1.f;
                const float bi = a.bias ? a.bias[m] : 0.f;
                const long long row = outb + (long long)m * N;
                float s0 = 0.f, s1 = 0.f;
#pragma unroll
                for (int nb = 0; nb < 4; ++nb) {
                    const float dg = bf16_round(acc[nb][i]);
                    const float hv = __bfloat162float(a.h[row + 32 * nb]);
                    const GeluParts gp = gelu_parts(fmaf(hv, sc, bi));
                    const float dz = dg * (gp.cdf + gp.zpdf);
                    a.out0[row + 32 * nb] = __float2bfloat16(dz * sc);
                    s0 = fmaf(dz, hv, s0);
                    s1 += dz;
                }
#pragma unroll
                for (int off = 16; off >= 1; off >>= 1) {     // sum over the 32 columns of this half
                    s0 += __shfl_xor(s0, off);
                    s1 += __shfl_xor(s1, off);
                }
                if (r == 0) {
                    const long long pi = ((long long)b * a.ntiles + tile) * M + m;
                    a.part0[pi] = s0;
                    a.part1[pi] = s1;
                }
            }
        }
    }
}

template <int MODE, int K>
int launch(const PwArgs& a, int B, hipStream_t st) {
    const size_t lds = (size_t)K * 256;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)pw_gemm_gelu<MODE, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL((pw_gemm_gelu<MODE, K>), dim3(a.ntiles, B), dim3(256), lds, st, a);
    return launch_status();
}

}  // namespace

extern "C" int vfm_pw_gemm_gelu(const void* A, const void* X, const float* scale, const float* bias,
                                const void* h, void* out0, void* out1, float* part0, float* part1, int mode,
                                int B, int M, int K, int N, void* stream) {
    if (!A || !X || B <= 0 || M <= 0 || N <= 0) return VFM_ERR_ARGS;
    if (M % (32 * WAVES) != 0 || N % NT != 0 || (K != 128 && K != 256 && K != 512)) return VFM_NO_KERNEL;
    if (mode == 0 && !out1) return VFM_ERR_ARGS;
    if (mode == 1 && (!h || !out0 || !part0 || !part1)) return VFM_ERR_ARGS;
    if (mode != 0 && mode != 1) return VFM_ERR_ARGS;
    PwArgs a;
    a.A = static_cast<const __hip_bfloat16*>(A);
    a.X = static_cast<const __hip_bfloat16*>(X);
    a.scale = scale;
    a.bias = bias;
    a.h = static_cast<const __hip_bfloat16*>(h);
    a.out0 = static_cast<__hip_bfloat16*>(out0);
    a.out1 = static_cast<__hip_bfloat16*>(out1);
    a.part0 = part0;
    a.part1 = part1;
    a.M = M;
    a.N = N;
    a.ntiles = N / NT;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (mode == 0) {
        switch (K) {
        case 128: return launch<0, 128>(a, B, st);
        case 256: return launch<0, 256>(a, B, st);
        default: return launch<0, 512>(a, B, st);
        }
    }
    switch (K) {
    case 128: return launch<1, 128>(a, B, st);
    case 256: return launch<1, 256>(a, B, st);
    default: return launch<1, 512>(a, B, st);
    }
}

extern "C" int vfm_pw_gemm_gelu_tiles(int N) { return (N > 0 && N % NT == 0) ? N / NT : VFM_NO_KERNEL; }
