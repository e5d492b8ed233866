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
// of 128 (8 waves: 4 row blocks of 32 x 2 column halves of 64), so X is read from HBM
// exactly once. A fragments come straight
// from global memory (the weight is tiny and L2-resident). v_mfma_f32_32x32x16_bf16:
// A lane l holds A[r][8h+j] (r = l&31, h = l>>5), B lane l holds B[8h+j][r], taken from the
// row-major X image with two ds_read_b64_tr_b16; C/D: col = l&31, row = (i&3)+8(i>>2)+4h.
//
// Status: parity-tested (tests/test_pwgemm_gpu.py); mode 1 runs the backward of the b5
// (C=128) ConvNeXt layers (torch_utils/ops/decoder_hip.py _ConvNeXtMLP); mode 0 is kept for
// the other widths' future use (the forward at C=128 is mlp_fwd below). Measured
// at batch 32 (tools_dev/pwbench.py, MI355X) against hipBLASLt bmm + the GELU row kernels:
//   C=128 @256^2: fwd h+g 1.36 ms (unfused 1.64), fwd g only 1.05 ms, bwd 1.94 ms (2.08)
//   C=256 @128^2: fwd h+g 0.87 ms (0.87), g only 0.70 ms, bwd 1.18 ms (1.03)
//   C=512 @64^2:  fwd h+g 0.83 ms (0.62), g only 0.58 ms, bwd 1.01 ms (0.66)
// What moved it: per-row scale/bias staged in LDS instead of a dependent global load per
// row in the epilogue, the epilogue's h loads issued together right after the MFMAs (not
// before them: that kept them live across the loop and cost occupancy; one step ahead was
// slower still), 8 waves x 2 column blocks (4 waves/SIMD), lane-pair packing for 4-byte h
// loads and outputs. Backward at C=128 / 256^2 is now 1.82 ms. Staging whole output rows
// through LDS was slower. Next: find what still caps the epilogue (PMC VALU/wait counters).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int NT = 128;   // pixel columns per workgroup
constexpr int WAVES = 8;  // wave w: rows 32(w&3) of every 128-row M step, columns 64(w>>2)..+63
constexpr int NBW = 2;    // 32-column MFMA blocks per wave
constexpr int PT = 64;    // columns summed into one backward partial (one wave's share)

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

__device__ __forceinline__ uint32_t bf16_bits(float v) {
    const __hip_bfloat16 b = __float2bfloat16(v);
    return (uint32_t)__builtin_bit_cast(uint16_t, b);
}

// Registers i (even) and i+1 of a 32x32 accumulator are rows m and m+1 of the same column
// (the lane). Lane pairs (r, r+1) trade one value so that the even lane holds columns
// (r, r+1) of row m and the odd lane columns (r-1, r) of row m+1: one 4-byte access per lane
// instead of two 2-byte ones. Returns the packed bf16 pair this lane stores.
__device__ __forceinline__ uint32_t pair_pack(float vi, float vi1, bool odd) {
    const uint32_t send = bf16_bits(odd ? vi : vi1);
    const uint32_t x = (uint32_t)__shfl_xor((int)send, 1);
    return odd ? (x | (bf16_bits(vi1) << 16)) : (bf16_bits(vi) | (x << 16));
}

typedef float f2 __attribute__((ext_vector_type(2)));

// z * Phi(z) for two values on the packed-fp32 ALU (v_pk_fma / v_pk_mul: half the issue slots of
// the scalar form); the same operations and constants as gelu_parts (vfm_common.h), so the result
// is bit-identical to z * gelu_parts(z).cdf.
__device__ __forceinline__ f2 gelu2(f2 z) {
    const f2 x = z * 0.70710678118654752f;
    const f2 ax = {fabsf(x.x), fabsf(x.y)};
    const f2 d = __builtin_elementwise_fma(ax, f2{0.3275911f, 0.3275911f}, f2{1.f, 1.f});
    const f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f2 p = __builtin_elementwise_fma(t, f2{1.061405429f, 1.061405429f}, f2{-1.453152027f, -1.453152027f});
    p = __builtin_elementwise_fma(p, t, f2{1.421413741f, 1.421413741f});
    p = __builtin_elementwise_fma(p, t, f2{-0.284496736f, -0.284496736f});
    p = __builtin_elementwise_fma(p, t, f2{0.254829592f, 0.254829592f});
    const f2 arg = -(x * x) * 1.4426950408889634f;
    const f2 e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
    const f2 q = (0.5f * (p * t)) * e;
    const f2 cdf = {x.x < 0.f ? q.x : 1.f - q.x, x.y < 0.f ? q.y : 1.f - q.y};
    return z * cdf;
}

// packed bf16 pair (round to nearest even) and its two values back as fp32
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, bf16x2));     // one v_cvt_pk_bf16_f32
}
__device__ __forceinline__ f2 unpk_bf16(uint32_t v) { return f2{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)}; }

template <int MODE, int K>
__global__ __launch_bounds__(64 * WAVES, 2) void pw_gemm_gelu(PwArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y;
    const int tile = blockIdx.x;
    const int n0 = tile * NT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rw = wave & 3, cw = wave >> 2;
    const int M = a.M, N = a.N;

    const __hip_bfloat16* xb = a.X + (long long)b * K * N + n0;
#pragma unroll 4
    for (int i = tid; i < K * 16; i += 64 * WAVES) {
        const int row = i >> 4, ch = i & 15;
        const uint4 v = *reinterpret_cast<const uint4*>(xb + (long long)row * N + ch * 8);
        *reinterpret_cast<uint4*>(lds + swz(row, ch)) = v;
    }
    // per-row epilogue constants of this sample, read from LDS in the epilogue (a global load
    // per row there would put its latency on the critical path of every row)
    float* s_sc = reinterpret_cast<float*>(lds + K * 256);
    float* s_bi = s_sc + M;
    for (int i = tid; i < M; i += 64 * WAVES) {
        s_sc[i] = a.scale ? a.scale[(long long)b * M + i] : 1.f;
        s_bi[i] = a.bias ? a.bias[i] : 0.f;
    }
    __syncthreads();

    const int r = lane & 31, hh = lane >> 5;
    const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    // transposed-read byte offsets for k-step 0; rows advance by 16 per k-step (the XOR term
    // depends on row & 15 only, so the offset of k-step s is base + 16 * 256 * s)
    int tro[NBW][2];
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
        const int c0 = 4 * (NBW * cw + j) + 2 * g1 + (p >> 1);
        tro[j][0] = swz(8 * hh + q, c0) + 8 * (p & 1);
        tro[j][1] = swz(8 * hh + 4 + q, c0) + 8 * (p & 1);
    }

    const long long outb = (long long)b * M * N + n0 + 64 * cw + r;
    for (int mc = 0; mc < M; mc += 128) {
        const int m0 = mc + 32 * rw;
        const __hip_bfloat16* arow = a.A + (long long)(m0 + r) * K + 8 * hh;
        f32x16 acc[NBW];
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) acc[nb] = f32x16{};
        bf16x8 a0 = *reinterpret_cast<const bf16x8*>(arow);
        bf16x8 a1 = *reinterpret_cast<const bf16x8*>(arow + 16);
#pragma unroll
        for (int s = 0; s < K / 16; ++s) {
            const bf16x8 af = a0;
            a0 = a1;
            if (s + 2 < K / 16) a1 = *reinterpret_cast<const bf16x8*>(arow + 16 * (s + 2));
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(lds + tro[nb][0] + 4096 * s));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(lds + tro[nb][1] + 4096 * s));
                const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, __builtin_bit_cast(bf16x8, both),
                                                                  acc[nb], 0, 0, 0);
            }
        }

        const bool odd = r & 1;
        uint32_t hraw[MODE == 1 ? 8 : 1][NBW];     // packed pairs, see pair_pack
        if (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 16; i += 2)
#pragma unroll
                for (int nb = 0; nb < NBW; ++nb) {
                    const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * hh + (odd ? 1 : 0);
                    hraw[i / 2][nb] = *reinterpret_cast<const uint32_t*>(a.h + outb - (odd ? 1 : 0) +
                                                                         (long long)m * N + 32 * nb);
                }
        }
        // epilogue: register i of acc[nb] is row m0 + (i&3) + 8(i>>2) + 4hh, column n0 + 32nb + r
        if (MODE == 0) {
            const bool odd = r & 1;
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const int mA = m0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const long long rowst = outb - (odd ? 1 : 0) + (long long)(mA + (odd ? 1 : 0)) * N;
#pragma unroll
                for (int nb = 0; nb < NBW; ++nb) {
                    float hv[2], gv[2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        hv[t] = bf16_round(acc[nb][i + t]);
                        const float z = fmaf(hv[t], s_sc[mA + t], s_bi[mA + t]);
                        gv[t] = z * gelu_parts(z).cdf;
                    }
                    if (a.out0)
                        *reinterpret_cast<uint32_t*>(a.out0 + rowst + 32 * nb) = pair_pack(hv[0], hv[1], odd);
                    *reinterpret_cast<uint32_t*>(a.out1 + rowst + 32 * nb) = pair_pack(gv[0], gv[1], odd);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const int mA = m0 + (i & 3) + 8 * (i >> 2) + 4 * hh;      // row of register i; i+1 is mA+1
                float s0[2] = {0.f, 0.f}, s1[2] = {0.f, 0.f};
#pragma unroll
                for (int nb = 0; nb < NBW; ++nb) {
                    // unpack this lane's h for rows mA, mA+1 (column r)
                    const uint32_t own = hraw[i / 2][nb];
                    const uint32_t x = (uint32_t)__shfl_xor((int)(odd ? (own & 0xffffu) : (own >> 16)), 1);
                    const uint32_t hb0 = odd ? x : (own & 0xffffu);
                    const uint32_t hb1 = odd ? (own >> 16) : x;
                    float dhv[2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int m = mA + t;
                        const float sc = s_sc[m];
                        const float bi = s_bi[m];
                        const float hv = __uint_as_float((t ? hb1 : hb0) << 16);
                        const float dg = bf16_round(acc[nb][i + t]);
                        const GeluParts gp = gelu_parts(fmaf(hv, sc, bi));
                        const float dz = dg * (gp.cdf + gp.zpdf);
                        dhv[t] = dz * sc;
                        s0[t] = fmaf(dz, hv, s0[t]);
                        s1[t] += dz;
                    }
                    const uint32_t pk = pair_pack(dhv[0], dhv[1], odd);
                    *reinterpret_cast<uint32_t*>(a.out0 + outb - (odd ? 1 : 0) + (long long)(mA + (odd ? 1 : 0)) * N +
                                                 32 * nb) = pk;
                }
                // sums of the 4 values (s0, s1) x (rows mA, mA+1) over the 32 columns of this half:
                // two halving butterfly steps (lanes keep / send opposite halves of the set) leave
                // one value per lane, value q = 2 * bit4(r) + bit3(r), then three plain xor steps;
                // 4 lanes per half hold the totals (12 shuffles instead of 20, one store)
                float v0, v1;
                {
                    const bool up = r & 16;
                    const float k0 = up ? s1[0] : s0[0], k1 = up ? s1[1] : s0[1];
                    const float d0 = up ? s0[0] : s1[0], d1 = up ? s0[1] : s1[1];
                    v0 = k0 + __shfl_xor(d0, 16);
                    v1 = k1 + __shfl_xor(d1, 16);
                }
                {
                    const bool up = r & 8;
                    v0 = (up ? v1 : v0) + __shfl_xor(up ? v0 : v1, 8);
                }
#pragma unroll
                for (int off = 4; off >= 1; off >>= 1) v0 += __shfl_xor(v0, off);
                if ((r & 7) == 0) {
                    const long long pi = ((long long)b * a.ntiles + 2 * tile + cw) * M + mA + ((r >> 3) & 1);
                    ((r & 16) ? a.part1 : a.part0)[pi] = v0;
                }
            }
        }
    }
}

template <int MODE, int K>
int launch(const PwArgs& a, int B, hipStream_t st) {
    const size_t lds = (size_t)K * 256 + 8 * (size_t)a.M;
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)pw_gemm_gelu<MODE, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  K * 256 + 8 * 2048);
        attr[dv_attr] = true;
    }
    VFM_LAUNCH((pw_gemm_gelu<MODE, K>), dim3(a.N / NT, B), dim3(64 * WAVES), lds, st, a);
    return launch_status();
}


// ---------------------------------------------------------------------------------------
// Whole ConvNeXt MLP forward without autograd (the D phase's no-grad generator pass):
//   out = x_in + gamma * (bf16(W2 . g) + b2),  g = bf16(GELU(bf16(W1 . m) * s + b1))
// per sample, with the 4C hidden tensor never leaving the chip: for every 128-row chunk of
// the hidden dimension the workgroup computes h (GEMM 1, X = m from LDS), writes g as bf16
// into an LDS image laid out like the X image, and accumulates GEMM 2 (B operand = that g
// image) into the C x 128 output accumulators it keeps across the chunks. HBM traffic is
// m + x_in + out instead of ~21 C x P tensors for the unfused pointwise/GELU/pointwise/
// residual chain. C in {128, 256}.
struct MlpArgs {
    const __hip_bfloat16* W1;   // [4C, C]
    const __hip_bfloat16* m;    // [B, C, N]
    const float* s;             // [B, 4C] or null
    const float* b1;            // [4C] or null
    const __hip_bfloat16* W2;   // [C, 4C]
    const float* b2;            // [C] or null
    const float* gamma;         // [C] or null
    const __hip_bfloat16* xin;  // [B, C, N]
    __hip_bfloat16* out;        // [B, C, N]
    __hip_bfloat16* hout;       // [B, 4C, N] bf16(W1 . m) for the backward, or null
    __hip_bfloat16* gout;       // [B, 4C, N] g, or null
    __hip_bfloat16* yout;       // [B, C, N] bf16(W2 . g), or null
    int N;
};

// SAVE: the autograd forward, which also writes h and g for the backward (a separate instantiation,
// so the no-grad launches carry no dead stores and rocprofv3 reports the two apart)
template <int C, bool SAVE>
__global__ __launch_bounds__(64 * WAVES, 2) void mlp_fwd(MlpArgs a) {
    constexpr int M = 4 * C;
    constexpr int YB = C / 128;                 // 32-row output blocks per wave (1 or 2)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* gimg = lds + C * 256;        // [128 hidden rows][128 cols] bf16 image
    float* s_sc = reinterpret_cast<float*>(gimg + 128 * 256);
    float* s_bi = s_sc + M;
    float* s_b2 = s_bi + M;
    float* s_gm = s_b2 + C;
    const int b = blockIdx.y;
    const int n0 = blockIdx.x * NT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rw = wave & 3, cw = wave >> 2;
    const int N = a.N;

    const __hip_bfloat16* xb = a.m + (long long)b * C * N + n0;
#pragma unroll 4
    for (int i = tid; i < C * 16; i += 64 * WAVES) {
        const int row = i >> 4, ch = i & 15;
        *reinterpret_cast<uint4*>(lds + swz(row, ch)) =
            *reinterpret_cast<const uint4*>(xb + (long long)row * N + ch * 8);
    }
    for (int i = tid; i < M; i += 64 * WAVES) {
        s_sc[i] = a.s ? a.s[(long long)b * M + i] : 1.f;
        s_bi[i] = a.b1 ? a.b1[i] : 0.f;
    }
    for (int i = tid; i < C; i += 64 * WAVES) {
        s_b2[i] = a.b2 ? a.b2[i] : 0.f;
        s_gm[i] = a.gamma ? a.gamma[i] : 1.f;
    }
    __syncthreads();

    const int r = lane & 31, hh = lane >> 5;
    const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const bool odd = r & 1;
    int tro[NBW][2];
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
        const int c0 = 4 * (NBW * cw + j) + 2 * g1 + (p >> 1);
        tro[j][0] = swz(8 * hh + q, c0) + 8 * (p & 1);
        tro[j][1] = swz(8 * hh + 4 + q, c0) + 8 * (p & 1);
    }
    const long long base = (long long)b * C * N + n0 + 64 * cw + r - (odd ? 1 : 0);
    f32x16 accy[YB][NBW];
#pragma unroll
    for (int yb = 0; yb < YB; ++yb)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) accy[yb][nb] = f32x16{};

    for (int mc = 0; mc < M; mc += 128) {
        // GEMM 1: h rows mc + 32rw .. +31, this wave's 64 columns
        const int m0 = mc + 32 * rw;
        const __hip_bfloat16* arow = a.W1 + (long long)(m0 + r) * C + 8 * hh;
        f32x16 acc[NBW];
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) acc[nb] = f32x16{};
        bf16x8 p0 = *reinterpret_cast<const bf16x8*>(arow);
        bf16x8 p1 = *reinterpret_cast<const bf16x8*>(arow + 16);
#pragma unroll
        for (int st = 0; st < C / 16; ++st) {
            const bf16x8 af = p0;
            p0 = p1;
            if (st + 2 < C / 16) p1 = *reinterpret_cast<const bf16x8*>(arow + 16 * (st + 2));
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + tro[nb][0] + 4096 * st));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + tro[nb][1] + 4096 * st));
                const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, __builtin_bit_cast(bf16x8, both), acc[nb], 0, 0, 0);
            }
        }
        // first two W2 fragments of GEMM 2, in flight during the GELU epilogue
        const __hip_bfloat16* a2row = a.W2 + (long long)(32 * rw + r) * M + mc + 8 * hh;
        bf16x8 q0 = *reinterpret_cast<const bf16x8*>(a2row);
        bf16x8 q1 = *reinterpret_cast<const bf16x8*>(a2row + 16);
        // GELU epilogue into the g image (row = hidden row within the chunk, column = pixel): registers
        // i, i+1 are rows lr, lr+1 of column col = 64 cw + 32 nb + r, processed as a packed pair;
        // 16-bit LDS / global writes per row (no lane-pair exchange)
        __hip_bfloat16* hb = SAVE ? a.hout + ((long long)b * M + mc) * N + n0 : nullptr;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const int lr = 32 * rw + (i & 3) + 8 * (i >> 2) + 4 * hh;     // chunk-local row of register i
            const f2 sc = {s_sc[mc + lr], s_sc[mc + lr + 1]};
            const f2 bi = {s_bi[mc + lr], s_bi[mc + lr + 1]};
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
                const int col = 64 * cw + 32 * nb + r;
                const uint32_t hp = pk_bf16(acc[nb][i], acc[nb][i + 1]);
                const f2 g = gelu2(__builtin_elementwise_fma(unpk_bf16(hp), sc, bi));
                const uint32_t gp = pk_bf16(g.x, g.y);
                const int o = swz(lr, col >> 3) + 2 * (col & 7);
                const int o1 = swz(lr + 1, col >> 3) + 2 * (col & 7);
                *reinterpret_cast<uint16_t*>(gimg + o) = (uint16_t)gp;
                *reinterpret_cast<uint16_t*>(gimg + o1) = (uint16_t)(gp >> 16);
                if constexpr (SAVE) {   // saved for the backward; g goes out below
                    const unsigned ho = (unsigned)(lr * N + col);               // uniform base + 32-bit offset
                    *reinterpret_cast<uint16_t*>(hb + ho) = (uint16_t)hp;
                    *reinterpret_cast<uint16_t*>(hb + ho + (unsigned)N) = (uint16_t)(hp >> 16);
                }
            }
        }
        __syncthreads();
        if constexpr (SAVE) {
            // g for the backward straight from the LDS image: 16-B chunks, whole 256-B rows per
            // 16 threads (the register layout would need 4-B stores of lane pairs)
#pragma unroll
            for (int k = 0; k < 128 * 16 / (64 * WAVES); ++k) {
                const int q = tid + 64 * WAVES * k, row = q >> 4, ch = q & 15;
                *reinterpret_cast<uint4*>(a.gout + ((long long)b * M + mc + row) * N + n0 + 8 * ch) =
                    *reinterpret_cast<const uint4*>(gimg + swz(row, ch));
            }
        }
        // GEMM 2: y[c] += W2[c, mc : mc + 128] . g
#pragma unroll
        for (int yb = 0; yb < YB; ++yb) {
            const __hip_bfloat16* a2 = a2row + (long long)128 * yb * M;
            if (yb > 0) {
                q0 = *reinterpret_cast<const bf16x8*>(a2);
                q1 = *reinterpret_cast<const bf16x8*>(a2 + 16);
            }
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                const bf16x8 af = q0;
                q0 = q1;
                if (st + 2 < 8) q1 = *reinterpret_cast<const bf16x8*>(a2 + 16 * (st + 2));
#pragma unroll
                for (int nb = 0; nb < NBW; ++nb) {
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(gimg + tro[nb][0] + 4096 * st));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(gimg + tro[nb][1] + 4096 * st));
                    const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    accy[yb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, __builtin_bit_cast(bf16x8, both),
                                                                           accy[yb][nb], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // out = x_in + gamma * (bf16(y) + b2); all residual loads are issued before the first store
    // (CDNA4 vmcnt counts stores, so interleaving would serialise every load behind them)
#pragma unroll
    for (int yb = 0; yb < YB; ++yb) {
        uint32_t xraw[8][NBW];
#pragma unroll
        for (int i = 0; i < 16; i += 2)
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
                const int cme = 32 * (rw + 4 * yb) + (i & 3) + 8 * (i >> 2) + 4 * hh + (odd ? 1 : 0);
                xraw[i / 2][nb] = *reinterpret_cast<const uint32_t*>(a.xin + base + (long long)cme * N + 32 * nb);
            }
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const int cA = 32 * (rw + 4 * yb) + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const int cme = cA + (odd ? 1 : 0);
            const float bb0 = s_b2[cA], bb1 = s_b2[cA + 1], gg0 = s_gm[cA], gg1 = s_gm[cA + 1];
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
                const uint32_t own = xraw[i / 2][nb];
                const uint32_t x = (uint32_t)__shfl_xor((int)(odd ? (own & 0xffffu) : (own >> 16)), 1);
                const float xv0 = __uint_as_float((odd ? x : (own & 0xffffu)) << 16);
                const float xv1 = __uint_as_float((odd ? (own >> 16) : x) << 16);
                const float y0 = bf16_round(accy[yb][nb][i]), y1 = bf16_round(accy[yb][nb][i + 1]);
                const float o0 = fmaf(gg0, y0 + bb0, xv0);
                const float o1 = fmaf(gg1, y1 + bb1, xv1);
                *reinterpret_cast<uint32_t*>(a.out + base + (long long)cme * N + 32 * nb) = pair_pack(o0, o1, odd);
                if (a.yout)
                    *reinterpret_cast<uint32_t*>(a.yout + base + (long long)cme * N + 32 * nb) = pair_pack(y0, y1, odd);
            }
        }
    }
}
template <int C, bool SAVE>
void launch_mlp(const MlpArgs& a, int B, size_t lds, hipStream_t st) {
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)mlp_fwd<C, SAVE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr[dv_attr] = true;
    }
    VFM_LAUNCH((mlp_fwd<C, SAVE>), dim3(a.N / NT, B), dim3(64 * WAVES), lds, st, a);
}
}  // namespace

extern "C" int vfm_pw_gemm_gelu(const void* A, const void* X, const float* scale, const float* bias,
                                const void* h, void* out0, void* out1, float* part0, float* part1, int mode,
                                int B, int M, int K, int N, void* stream) {
    if (!A || !X || B <= 0 || M <= 0 || N <= 0) return VFM_ERR_ARGS;
    if (M % 128 != 0 || M > 2048 || N % NT != 0 || (K != 128 && K != 256 && K != 512)) return VFM_NO_KERNEL;
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
    a.ntiles = N / PT;
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

extern "C" int vfm_pw_gemm_gelu_tiles(int N) { return (N > 0 && N % NT == 0) ? N / PT : VFM_NO_KERNEL; }

extern "C" int vfm_convnext_mlp_fwd(const void* W1, const void* m, const float* s, const float* b1, const void* W2,
                                    const float* b2, const float* gamma, const void* xin, void* out, void* hout,
                                    void* gout, void* yout, int B, int C, int N, void* stream) {
    if (!W1 || !m || !W2 || !xin || !out || B <= 0 || N <= 0) return VFM_ERR_ARGS;
    if ((hout == nullptr) != (gout == nullptr)) return VFM_ERR_ARGS;
    if ((C != 128 && C != 256) || N % NT != 0) return VFM_NO_KERNEL;
    MlpArgs a;
    a.W1 = static_cast<const __hip_bfloat16*>(W1);
    a.m = static_cast<const __hip_bfloat16*>(m);
    a.s = s;
    a.b1 = b1;
    a.W2 = static_cast<const __hip_bfloat16*>(W2);
    a.b2 = b2;
    a.gamma = gamma;
    a.xin = static_cast<const __hip_bfloat16*>(xin);
    a.out = static_cast<__hip_bfloat16*>(out);
    a.hout = static_cast<__hip_bfloat16*>(hout);
    a.gout = static_cast<__hip_bfloat16*>(gout);
    a.yout = static_cast<__hip_bfloat16*>(yout);
    a.N = N;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t lds = (size_t)C * 256 + 128 * 256 + 8 * 4 * (size_t)C + 8 * (size_t)C;
    const bool save = hout != nullptr;
    if (C == 128) {
        if (save) launch_mlp<128, true>(a, B, lds, st);
        else launch_mlp<128, false>(a, B, lds, st);
    } else {
        if (save) launch_mlp<256, true>(a, B, lds, st);
        else launch_mlp<256, false>(a, B, lds, st);
    }
    return launch_status();
}
