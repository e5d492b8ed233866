// Depthwise K x K conv (K = 3, 5, 7; stride 1, pad (K-1)/2) of bf16 planes on the MFMA cores
// (the ConvNeXt layers' dwconv of the bf16 decoder blocks, reference convnext_utils.py:121-124 /
// :243, nn.Conv2d(groups=C) under bf16 autocast: bf16 input and weight, fp32 accumulation; and its
// data gradient, the same conv with the 180-degree-rotated taps).
//
// A depthwise conv has K*K MACs per output and no reuse across channels, so on the vector ALU it
// is VALU-bound (49 FMAs per bf16 output at K = 7, ~0.2 of HBM for the row-streaming kernel in
// decoder.hip). Here each kernel row ky is a banded matrix product on v_mfma_f32_16x16x32_bf16:
//
//   out[y0 + n][x0 + i] += sum_j  A_ky[i][j] * X[y0 + n + ky - P][x0 - 8 + j],
//   A_ky[i][j] = w[ky][j - i - 8 + P]  (0 <= j - i - 8 + P < K, else 0),  i, n < 16, j < 32,
//
// so a 16 x 16 output tile is K MFMAs (K * 16 of their 32 k-slots are nonzero: the MFMA pipe has
// ~20x the needed rate, the kernel is left HBM-bound). The band origin x0 - 8 keeps every B fragment
// (8 consecutive input columns of one row) a 16-B aligned read. One wave owns a 16-row x XW-column
// output block of one plane: it stages the 16 + K - 1 input rows x (XW + 16) columns in LDS once
// (16-B loads, zero halo, row stride an odd multiple of 16 B so the 16 row-lanes of a fragment read
// hit distinct bank groups), builds its K A-fragments from the channel's taps (staged through LDS),
// and runs XW / 16 tiles x K MFMAs; a wave walks up to 4 such row blocks down the plane with the next
// block's loads in flight during the current block's MFMAs. Output: lane l holds
// out[y0 + (l & 15)][x0 + 16 s + 4 (l >> 4) + r], r < 4 -> one 8-B store per tile (+ the fp32 noise
// plane of the legacy noise path when given).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVES = 4;
constexpr int ROWS = 22;                  // 16 + K - 1 for K <= 7

struct DwmArgs {
    const __hip_bfloat16* x;
    const float* w;                       // [C, K, K] fp32 (rounded to bf16 here, as autocast does)
    const float* bias;                    // [C] or null
    const float* noise;                   // [H, W] fp32 added to every channel (legacy noise) or null
    __hip_bfloat16* y;
    int B, C, H, W, XW, nyb, nxs, rb;     // rb: 16-row blocks per wave
    long long units;
};

__device__ __forceinline__ uint16_t bf16_bits(float v) { return __builtin_bit_cast(uint16_t, __float2bfloat16(v)); }

template <int K, int XW>
__global__ __launch_bounds__(64 * WAVES) void dwm_fwd(DwmArgs a) {
    constexpr int P = (K - 1) / 2;
    constexpr int NQ = XW / 8 + 2;                          // 16-B chunks per staged row
    constexpr int RS = ((NQ * 16 / 16) | 1) * 16;           // row stride (bytes): odd multiple of 16
    constexpr int NR = 16 + K - 1;
    constexpr int NL = (NR * NQ + 63) / 64;                 // staging loads per lane per row block
    __shared__ __attribute__((aligned(16))) unsigned char lds[WAVES][ROWS * RS];
    __shared__ float taps[WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long unit = (long long)blockIdx.x * WAVES + wave;
    if (unit >= a.units) return;                            // wave-uniform; no block-level barrier below
    const int xs = (int)(unit % a.nxs);
    long long t = unit / a.nxs;
    const int ybg = (int)(t % a.nyb);                       // group of rb row blocks
    t /= a.nyb;
    const int c = (int)(t % a.C);
    const int x0 = xs * XW;
    const long long plane = t * (long long)a.H * a.W;       // (b * C + c) * H * W
    const __hip_bfloat16* xp = a.x + plane;
    unsigned char* img = lds[wave];

    // staging of row block y0: rows y0 - P .. y0 + 15 + K - 1 - P, columns x0 - 8 .. x0 + XW + 7,
    // zero outside the plane; loads go to registers first so the next block's are in flight while
    // the current block computes
    uint4 st[NL];
    auto fetch = [&](int y0) {
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int q = lane + 64 * u;
            const int r = q / NQ, ch = q - r * NQ;
            const int yy = y0 - P + r, xx = x0 - 8 + 8 * ch;
            st[u] = make_uint4(0, 0, 0, 0);
            if (q < NR * NQ && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
                st[u] = *reinterpret_cast<const uint4*>(xp + (long long)yy * a.W + xx);
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int q = lane + 64 * u;
            const int r = q / NQ, ch = q - r * NQ;
            if (q < NR * NQ) *reinterpret_cast<uint4*>(img + r * RS + 16 * ch) = st[u];
        }
    };
    const int yb0 = ybg * a.rb;
    const int nblk = min(a.rb, (a.H + 15) / 16 - yb0);
    fetch(16 * yb0);

    // the channel's taps, one per lane, through LDS (one global load per lane instead of 8 K)
    if (lane < K * K) taps[wave][lane] = a.w[(long long)c * K * K + lane];
    __builtin_amdgcn_wave_barrier();
    // A fragments: lane l holds A_ky[i = l & 15][j = 8 (l >> 4) + e], e < 8
    const int i = lane & 15, g = lane >> 4;
    bf16x8 af[K];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        uint32_t u[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
            uint32_t h2 = 0;
#pragma unroll
            for (int hlf = 0; hlf < 2; ++hlf) {
                const int kx = 8 * g + 2 * e2 + hlf - i - 8 + P;
                const float wv = (kx >= 0 && kx < K) ? taps[wave][ky * K + kx] : 0.f;
                h2 |= (uint32_t)bf16_bits(wv) << (16 * hlf);
            }
            u[e2] = h2;
        }
        af[ky] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    }
    const float bias = a.bias ? a.bias[c] : 0.f;
    const int n = lane & 15;                                // output row of this lane (B / C column)

    for (int kb = 0; kb < nblk; ++kb) {
        const int y0 = 16 * (yb0 + kb);
        put();                                              // after the previous block's fragment reads
        if (kb + 1 < nblk) fetch(y0 + 16);
        __builtin_amdgcn_wave_barrier();
        const int oy = y0 + n;
        __hip_bfloat16* yp = a.y + plane + (long long)oy * a.W + x0 + 4 * g;
        const float* np = a.noise ? a.noise + (long long)oy * a.W + x0 + 4 * g : nullptr;
#pragma unroll
        for (int s = 0; s < XW / 16; ++s) {
            f32x4 acc = {bias, bias, bias, bias};
            if (np && oy < a.H) {
                const float4 nz = *reinterpret_cast<const float4*>(np + 16 * s);
                acc[0] += nz.x; acc[1] += nz.y; acc[2] += nz.z; acc[3] += nz.w;
            }
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(img + (n + ky) * RS + 16 * (2 * s + g));
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ky], b, acc, 0, 0, 0);
            }
            if (oy < a.H) {
                const uint2 o = make_uint2((uint32_t)bf16_bits(acc[0]) | ((uint32_t)bf16_bits(acc[1]) << 16),
                                           (uint32_t)bf16_bits(acc[2]) | ((uint32_t)bf16_bits(acc[3]) << 16));
                *reinterpret_cast<uint2*>(yp + 16 * s) = o;
            }
        }
    }
}

template <int K>
int dwm_launch(DwmArgs& a, hipStream_t st) {
    const long long blocks = (a.units + WAVES - 1) / WAVES;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    if (a.XW == 64) hipLaunchKernelGGL((dwm_fwd<K, 64>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
    else hipLaunchKernelGGL((dwm_fwd<K, 16>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
    return launch_status();
}

}  // namespace

// y = dwconv(x, w) + bias on bf16 NCHW planes via MFMA (see the header). VFM_NO_KERNEL for shapes it
// does not cover (W % 16, pad != (K - 1) / 2, K not in {3, 5, 7}, misaligned pointers): the caller
// then uses vfm_dwconv2d_fwd.
extern "C" int vfm_dwconv2d_fwd_mfma(const void* x, const float* w, const float* bias, const float* noise, void* y,
                                     int B, int C, int H, int W, int K, int pad, void* stream) {
    if (!x || !w || !y || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    if ((K != 3 && K != 5 && K != 7) || pad != (K - 1) / 2 || W % 16) return VFM_NO_KERNEL;
    if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)noise) % 16) return VFM_NO_KERNEL;
    DwmArgs a;
    a.x = (const __hip_bfloat16*)x; a.w = w; a.bias = bias; a.noise = noise; a.y = (__hip_bfloat16*)y;
    a.B = B; a.C = C; a.H = H; a.W = W;
    a.XW = W % 64 == 0 ? 64 : 16;
    const int rows16 = (H + 15) / 16;
    a.rb = rows16 < 4 ? rows16 : 4;                        // up to 64 output rows per wave
    a.nyb = (rows16 + a.rb - 1) / a.rb;
    a.nxs = W / a.XW;
    a.units = (long long)B * C * a.nyb * a.nxs;
    hipStream_t st = (hipStream_t)stream;
    switch (K) {
    case 3: return dwm_launch<3>(a, st);
    case 5: return dwm_launch<5>(a, st);
    default: return dwm_launch<7>(a, st);
    }
}
