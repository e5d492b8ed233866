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
// (16-B loads, zero halo, row stride chosen so each ds_read_b128 lane group of a fragment read hits
// 16 distinct 16-B bank slots), builds its K A-fragments from the channel's taps (staged through LDS),
// and runs XW / 16 tiles x K MFMAs; a wave walks up to 4 such row blocks down the plane with the next
// block's loads in flight during the current block's MFMAs. Output: lane l holds
// out[y0 + (l & 15)][x0 + 16 s + 4 (l >> 4) + r], r < 4 -> one 8-B store per tile (+ the fp32 noise
// plane of the legacy noise path, and / or a residual tensor (the data gradient's other branch),
// when given). With npart (the data gradient of a legacy-noise layer), each wave also writes
// npart[unit] = sum over its output positions of x[b, c, y, x] * nplane[y, x] from the staged input
// rows: the noise strength's gradient sum_{b,c,y,x} dY * noise_plane without another pass over dY.
#include "vfm_common.h"

#include <cstdlib>
#include <type_traits>

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
    const __hip_bfloat16* res;            // [B, C, H, W] bf16 added before the output rounding, or null
    const float* nplane;                  // [H, W] fp32: with npart, sum x * nplane per wave (see below)
    float* npart;                         // [units] or null
    // [units][4] or null: the wave's GroupNorm statistics of its stored (bf16-rounded) outputs, {count, shift,
    // sum (y - shift), sum (y - shift)^2} with shift = the wave's first output (group_norm_fwd_stats merges them)
    float* gstat;
    __hip_bfloat16* y;
    int B, C, H, W, XW, nyb, nxs, rb;     // rb: 16-row blocks per wave
    int flip;                             // taps read rotated by 180 degrees (the data gradient)
    long long units;
};

// two floats -> packed bf16 pair (RNE, element 0 low), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk_bf16(float a0, float a1) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(vfm_f2{a0, a1}, vfm_bf16x2));
}

template <int K, int XW, bool GS>
__global__ __launch_bounds__(64 * WAVES) void dwm_fwd(DwmArgs a) {
    constexpr int P = (K - 1) / 2;
    constexpr int NQ = XW / 8 + 2;                          // 16-B chunks per staged row
    // row stride: R 16-B slots with R = 2 (mod 4), R >= NQ. The B-fragment ds_read_b128 of lane
    // (n = l & 15, g = l >> 4) starts at slot R n + 2 s + g; with R = 2 (mod 4) the 16 lanes of each
    // of its four lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) land on 16 distinct slots of
    // the 256-B bank row (conflict-free; the odd strides used before were 2-way), and the staging
    // stores stay contiguous when R = NQ.
    constexpr int RS = (NQ + (6 - NQ % 4) % 4) * 16;
    constexpr int NR = 16 + K - 1;
    constexpr int NL = (NR * NQ + 63) / 64;                 // staging loads per lane per row block
    __shared__ __attribute__((aligned(16))) unsigned char lds[WAVES][ROWS * RS];
    constexpr int TOFF = 23, TROW = 48;                     // padded tap row: kx + TOFF - P in [0, 47)
    __shared__ float taps[WAVES][K * TROW];
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
    // per staging slot u (loop-invariant): its row r - P relative to y0 (or a large negative value when
    // the slot is unused or its columns lie outside the plane), its 16-B chunk and its LDS offset
    // (srow packed with the chunk index: srow * 16 + ch, two registers per slot with slds)
    // D staging register sets: the non-GS forms (the data gradient) keep two row blocks' loads in flight
    // (108 -> ~124 VGPRs, still 4 waves per SIMD); the GS form one (128 VGPRs)
    constexpr int D = GS ? 1 : 2;
    uint4 st[D][NL];
    int srow[NL], slds[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int q = lane + 64 * u;
        const int r = q / NQ, ch = q - r * NQ;
        const int xx = x0 - 8 + 8 * ch;
        const bool ok = q < NR * NQ && xx >= 0 && xx < a.W;
        srow[u] = (ok ? r - P : -(1 << 24)) * 16 + ch;
        slds[u] = q < NR * NQ ? r * RS + 16 * ch : -1;
    }
    auto fetch = [&](auto bc, int y0) {
        constexpr int BF = decltype(bc)::value;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int yy = y0 + (srow[u] >> 4);
            st[BF][u] = make_uint4(0, 0, 0, 0);
            if ((unsigned)yy < (unsigned)a.H)
                st[BF][u] = *reinterpret_cast<const uint4*>(xp + (long long)yy * a.W + x0 - 8 + 8 * (srow[u] & 15));
        }
    };
    auto put = [&](auto bc) {
        constexpr int BF = decltype(bc)::value;
#pragma unroll
        for (int u = 0; u < NL; ++u)
            if (slds[u] >= 0) *reinterpret_cast<uint4*>(img + slds[u]) = st[BF][u];
    };
    constexpr std::integral_constant<int, 0> buf0{};
    constexpr std::integral_constant<int, D - 1> buf1{};
    const int yb0 = ybg * a.rb;
    const int nblk = min(a.rb, (a.H + 15) / 16 - yb0);
    fetch(buf0, 16 * yb0);
    if constexpr (D == 2) {
        if (nblk > 1) fetch(buf1, 16 * (yb0 + 1));
    }

    // the channel's taps through LDS as zero-padded rows: tp[ky][kx + TOFF] (one global load per lane
    // instead of 8 K), so a lane's 8 band values of a kernel row are 8 consecutive entries, read without
    // range tests (the band's kx = 8 g + e - i - 8 + P spans -23 + P .. 23 + P over the wave)
    float* tp = taps[wave];
#pragma unroll
    for (int t = lane; t < K * TROW; t += 64) tp[t] = 0.f;
    __builtin_amdgcn_wave_barrier();
    if (lane < K * K) {
        const int ky = lane / K, kx = lane - ky * K;
        tp[ky * TROW + kx + TOFF - P] = a.w[(long long)c * K * K + (a.flip ? K * K - 1 - lane : lane)];
    }
    __builtin_amdgcn_wave_barrier();
    // A fragments: lane l holds A_ky[i = l & 15][j = 8 (l >> 4) + e], e < 8 (taps rounded to bf16, RNE)
    const int i = lane & 15, g = lane >> 4;
    const int tb = 8 * g - i - 8 + TOFF;                    // row entry of e = 0
    bf16x8 af[K];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        const float* row = tp + ky * TROW + tb;
        uint32_t u[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) u[e2] = pk_bf16(row[2 * e2], row[2 * e2 + 1]);
        af[ky] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    }
    const float bias = a.bias ? a.bias[c] : 0.f;
    const int n = lane & 15;                                // output row of this lane (B / C column)
    float ndot = 0.f;
    float g_sh = 0.f, g_s1 = 0.f, g_s2 = 0.f, g_n = 0.f;    // GroupNorm statistics (GS: a.gstat)

    auto body = [&](auto bc, int kb) {
        const int y0 = 16 * (yb0 + kb);
        put(bc);                                            // after the previous block's fragment reads
        if (kb + D < nblk) fetch(bc, y0 + 16 * D);
        __builtin_amdgcn_wave_barrier();
        const int oy = y0 + n;
        __hip_bfloat16* yp = a.y + plane + (long long)oy * a.W + x0 + 4 * g;
        const float* np = a.noise ? a.noise + (long long)oy * a.W + x0 + 4 * g : nullptr;
        const __hip_bfloat16* rp = a.res ? a.res + plane + (long long)oy * a.W + x0 + 4 * g : nullptr;
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
            if (rp && oy < a.H) {          // residual-branch gradient (the layer's other use of x)
                const uint2 rv = *reinterpret_cast<const uint2*>(rp + 16 * s);
                acc[0] += __uint_as_float(rv.x << 16); acc[1] += __uint_as_float(rv.x & 0xffff0000u);
                acc[2] += __uint_as_float(rv.y << 16); acc[3] += __uint_as_float(rv.y & 0xffff0000u);
            }
            const uint2 o = make_uint2(pk_bf16(acc[0], acc[1]), pk_bf16(acc[2], acc[3]));   // 2 v_cvt_pk_bf16_f32
            if constexpr (GS) {
                // statistics of the rounded outputs; the shift is lane 0's first value (row y0 >= 0 is in the plane)
                const float v[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                                    __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
                if (kb == 0 && s == 0) g_sh = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                  __builtin_bit_cast(int, v[0])));
                if (oy < a.H) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float d = v[r] - g_sh;
                        g_s1 += d;
                        g_s2 = fmaf(d, d, g_s2);
                    }
                    g_n += 4.f;
                }
            }
            if (oy < a.H) {
                *reinterpret_cast<uint2*>(yp + 16 * s) = o;
                if (a.npart) {     // input at the output position: staged row n + P, column 8 + 16 s + 4 g
                    const uint2 xv = *reinterpret_cast<const uint2*>(img + (n + P) * RS + 16 + 32 * s + 8 * g);
                    const float4 pl = *reinterpret_cast<const float4*>(a.nplane + (long long)oy * a.W + x0 +
                                                                       16 * s + 4 * g);
                    ndot = fmaf(__uint_as_float(xv.x << 16), pl.x, ndot);
                    ndot = fmaf(__uint_as_float(xv.x & 0xffff0000u), pl.y, ndot);
                    ndot = fmaf(__uint_as_float(xv.y << 16), pl.z, ndot);
                    ndot = fmaf(__uint_as_float(xv.y & 0xffff0000u), pl.w, ndot);
                }
            }
        }
    };
    for (int kb = 0; kb < nblk; kb += D) {
        body(buf0, kb);
        if constexpr (D == 2) {
            if (kb + 1 < nblk) body(buf1, kb + 1);
        }
    }
    if (a.npart) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) ndot += __shfl_xor(ndot, m);
        if (lane == 0) a.npart[unit] = ndot;
    }
    if constexpr (GS) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            g_s1 += __shfl_xor(g_s1, m);
            g_s2 += __shfl_xor(g_s2, m);
            g_n += __shfl_xor(g_n, m);
        }
        if (lane == 0) *reinterpret_cast<float4*>(a.gstat + 4 * unit) = make_float4(g_n, g_sh, g_s1, g_s2);
    }
}

template <int K>
int dwm_launch(DwmArgs& a, hipStream_t st) {
    const long long blocks = (a.units + WAVES - 1) / WAVES;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    if (a.gstat) {
        if (a.XW == 64) VFM_LAUNCH((dwm_fwd<K, 64, true>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
        else VFM_LAUNCH((dwm_fwd<K, 16, true>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
    } else {
        if (a.XW == 64) VFM_LAUNCH((dwm_fwd<K, 64, false>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
        else VFM_LAUNCH((dwm_fwd<K, 16, false>), dim3((unsigned)blocks), dim3(64 * WAVES), 0, st, a);
    }
    return launch_status();
}


// ---- weight gradient -------------------------------------------------------------------------
//   dW[ky][kx] = sum_{b, y, x} dY[y][x] X[y + ky - P][x + kx - P],   db = sum dY
// per 32-row x 16-column dY tile and kernel row ky, with j over the 32 input columns x0 - 8 + j:
//   T_ky[i][j] = sum_{n < 32} dY[y0 + n][x0 + i] X[y0 + n + ky - P][x0 - 8 + j]   (one MFMA per j-half)
//   dW[ky][kx] = sum_i T_ky[i][i + kx + 8 - P]                                     (diagonals, once per wave)
// Both operands run along the rows (the MFMA k dimension), i.e. against the memory layout: the
// fragments come from the LDS images with ds_read_b64_tr_b16 (the hardware transpose read). T_ky
// accumulates in registers over all tiles of the wave's bands; at the end the accumulators go to LDS
// and 49 lanes sum the diagonals. One fp32 partial [K K + 1] per wave (host sums in a fixed order).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct DwmBwArgs {
    const __hip_bfloat16* x;
    const __hip_bfloat16* dy;
    float* partial;                       // [tiles, C, K K + 1]
    int B, C, H, W, nyb, nxs, tiles, per; // per: bands per wave; bands per channel = B nyb nxs
};

__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* lo, const unsigned char* hi) {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo);
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int K, int XW>
__global__ __launch_bounds__(64 * 2) void dwm_bwd_w(DwmBwArgs a) {
    constexpr int P = (K - 1) / 2;
    constexpr int RSD = ((XW * 2 / 16) | 1) * 16;           // dY image row stride (bytes)
    constexpr int NQX = XW / 8 + 2;
    constexpr int RSX = ((NQX * 16 / 16) | 1) * 16;         // X image row stride
    constexpr int NRX = 32 + K - 1;
    constexpr int QD = 32 * XW / 8, QX = NRX * NQX;          // 16-B chunks per band
    constexpr int LD = (QD + 63) / 64, LX = (QX + 63) / 64;
    constexpr int IMG = 32 * RSD + NRX * RSX;
    constexpr int SCR = K * 16 * 32 * 4;                     // diagonal scratch (end of the wave)
    constexpr int AREA = ((IMG > SCR ? IMG : SCR) + 15) / 16 * 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][AREA];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long wg = (long long)blockIdx.x * 2 + wave;
    if (wg >= (long long)a.C * a.tiles) return;             // wave-uniform
    const int c = (int)(wg / a.tiles), tile = (int)(wg - (long long)c * a.tiles);
    unsigned char* dimg = lds[wave];
    unsigned char* ximg = dimg + 32 * RSD;
    const int nbands = a.B * a.nyb * a.nxs;
    const int band0 = tile * a.per, band1 = min(nbands, band0 + a.per);

    uint4 sd[LD], sx[LX];
    auto fetch = [&](int band) {
        const int xs = band % a.nxs;
        const int t = band / a.nxs;
        const int yb = t % a.nyb, b = t / a.nyb;
        const int x0 = xs * XW, y0 = yb * 32;
        const long long plane = ((long long)b * a.C + c) * a.H * a.W;
#pragma unroll
        for (int u = 0; u < LD; ++u) {
            const int q = lane + 64 * u, r = q / (XW / 8), ch = q - r * (XW / 8);
            sd[u] = make_uint4(0, 0, 0, 0);
            if (q < QD && y0 + r < a.H)
                sd[u] = *reinterpret_cast<const uint4*>(a.dy + plane + (long long)(y0 + r) * a.W + x0 + 8 * ch);
        }
#pragma unroll
        for (int u = 0; u < LX; ++u) {
            const int q = lane + 64 * u, r = q / NQX, ch = q - r * NQX;
            const int yy = y0 - P + r, xx = x0 - 8 + 8 * ch;
            sx[u] = make_uint4(0, 0, 0, 0);
            if (q < QX && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
                sx[u] = *reinterpret_cast<const uint4*>(a.x + plane + (long long)yy * a.W + xx);
        }
    };
    float dbs = 0.f;
    auto put = [&]() {
#pragma unroll
        for (int u = 0; u < LD; ++u) {
            const int q = lane + 64 * u, r = q / (XW / 8), ch = q - r * (XW / 8);
            if (q < QD) {
                *reinterpret_cast<uint4*>(dimg + r * RSD + 16 * ch) = sd[u];
                const uint32_t w4[4] = {sd[u].x, sd[u].y, sd[u].z, sd[u].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) dbs += __uint_as_float(w4[e] << 16) + __uint_as_float(w4[e] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int u = 0; u < LX; ++u) {
            const int q = lane + 64 * u, r = q / NQX, ch = q - r * NQX;
            if (q < QX) *reinterpret_cast<uint4*>(ximg + r * RSX + 16 * ch) = sx[u];
        }
    };

    f32x4 acc[K][2];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) acc[ky][0] = acc[ky][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    if (band0 < band1) fetch(band0);
    for (int band = band0; band < band1; ++band) {
        put();                                              // after the previous band's fragment reads
        if (band + 1 < band1) fetch(band + 1);
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int s = 0; s < XW / 16; ++s) {
            // A[i][n] = dY[n][16 s + i]: image rows 8 g + q4 (+4), columns 16 s + 4 p4
            const bf16x8 af = tr_frag(dimg + (8 * g + q4) * RSD + 2 * (16 * s + 4 * p4),
                                      dimg + (8 * g + 4 + q4) * RSD + 2 * (16 * s + 4 * p4));
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int jb = 0; jb < 2; ++jb) {
                    const int col = 2 * (16 * s + 16 * jb + 4 * p4);
                    const bf16x8 bfr = tr_frag(ximg + (ky + 8 * g + q4) * RSX + col,
                                               ximg + (ky + 8 * g + 4 + q4) * RSX + col);
                    acc[ky][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[ky][jb], 0, 0, 0);
                }
        }
    }
    // diagonals: lane holds T_ky[i = 4 g + r][j = 16 jb + (l & 15)]
    __builtin_amdgcn_wave_barrier();
    float* scr = reinterpret_cast<float*>(lds[wave]);       // [K][16][32]
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) scr[(ky * 16 + 4 * g + r) * 32 + 16 * jb + (lane & 15)] = acc[ky][jb][r];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) dbs += __shfl_xor(dbs, o, 64);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float* out = a.partial + ((long long)tile * a.C + c) * (K * K + 1);
    if (lane < K * K) {
        const int ky = lane / K, kx = lane - ky * K;
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += scr[(ky * 16 + i) * 32 + i + kx + 8 - P];
        out[lane] = t;
    } else if (lane == K * K) {
        out[lane] = dbs;
    }
}

template <int K>
int dwm_bw_launch(DwmBwArgs& a, int XW, hipStream_t st) {
    const long long waves = (long long)a.C * a.tiles;
    const long long blocks = (waves + 1) / 2;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    if (XW == 64) VFM_LAUNCH((dwm_bwd_w<K, 64>), dim3((unsigned)blocks), dim3(128), 0, st, a);
    else VFM_LAUNCH((dwm_bwd_w<K, 16>), dim3((unsigned)blocks), dim3(128), 0, st, a);
    return launch_status();
}

// bands per channel and bands per wave: ~16k waves over the whole grid
bool dwm_bw_plan(DwmBwArgs& a, int B, int C, int H, int W, int& XW) {
    XW = W % 64 == 0 ? 64 : 16;
    a.B = B; a.C = C; a.H = H; a.W = W;
    a.nyb = (H + 31) / 32;
    a.nxs = W / XW;
    const long long nb = (long long)B * a.nyb * a.nxs;
    if (nb > 0x7fffffffLL) return false;
    long long want = (16384 + C - 1) / C;                   // waves per channel
    if (want > nb) want = nb;
    a.per = (int)((nb + want - 1) / want);
    a.tiles = (int)((nb + a.per - 1) / a.per);
    return true;
}

bool dwm_plan(DwmArgs& a, int B, int C, int H, int W, int K, int pad) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return false;
    if ((K != 3 && K != 5 && K != 7) || pad != (K - 1) / 2 || W % 16) return false;
    a.B = B; a.C = C; a.H = H; a.W = W;
    a.XW = W % 64 == 0 ? 64 : 16;
    const int rows16 = (H + 15) / 16;
    // up to 4 row blocks (64 output rows) per wave. VFM_DWM_RB overrides the cap (A/B, profiles/r5_bi_dwm_rb.txt:
    // 8 or 16 blocks amortise the wave's prologue better but leave fewer waves: the plain form 6-19 % slower at
    // 256^2, the GS form 2 % faster at 8)
    static const int rb_cap = [] {
        const char* e = getenv("VFM_DWM_RB");
        const int v = e ? atoi(e) : 4;
        return v < 1 ? 1 : v;
    }();
    a.rb = rows16 < rb_cap ? rows16 : rb_cap;
    a.nyb = (rows16 + a.rb - 1) / a.rb;
    a.nxs = W / a.XW;
    a.units = (long long)B * C * a.nyb * a.nxs;
    return true;
}

}  // namespace

// y = dwconv(x, w) + bias on bf16 NCHW planes via MFMA (see the header). VFM_NO_KERNEL for shapes it
// does not cover (W % 16, pad != (K - 1) / 2, K not in {3, 5, 7}, misaligned pointers): the caller
// then uses vfm_dwconv2d_fwd. With npart (vfm_dwconv2d_fwd_mfma_units entries) and nplane [H, W] fp32:
// npart[u] = the wave's share of sum_{b, c, y, x} x[b, c, y, x] nplane[y, x].
extern "C" int vfm_dwconv2d_fwd_mfma_nz(const void* x, const float* w, const float* bias, const float* noise,
                                        const void* res, void* y, const float* nplane, float* npart, int B, int C,
                                        int H, int W, int K, int pad, int flip, void* stream) {
    if (!x || !w || !y || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    if (!npart != !nplane) return VFM_ERR_ARGS;
    DwmArgs a;
    if (!dwm_plan(a, B, C, H, W, K, pad)) return VFM_NO_KERNEL;
    if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)noise | (uintptr_t)res | (uintptr_t)nplane) % 16)
        return VFM_NO_KERNEL;
    a.x = (const __hip_bfloat16*)x; a.w = w; a.bias = bias; a.noise = noise; a.y = (__hip_bfloat16*)y;
    a.res = (const __hip_bfloat16*)res;
    a.nplane = nplane; a.npart = npart;
    a.gstat = nullptr;
    a.flip = flip != 0;
    hipStream_t st = (hipStream_t)stream;
    switch (K) {
    case 3: return dwm_launch<3>(a, st);
    case 5: return dwm_launch<5>(a, st);
    default: return dwm_launch<7>(a, st);
    }
}

// vfm_dwconv2d_fwd_mfma with the GroupNorm statistics of y: gstat [units][4] (vfm_dwconv2d_fwd_mfma_units; the
// units of a (sample, channel) plane are consecutive), consumed by vfm_group_norm_fwd_stats.
extern "C" int vfm_dwconv2d_fwd_mfma_gs(const void* x, const float* w, const float* bias, const float* noise, void* y,
                                        float* gstat, int B, int C, int H, int W, int K, int pad, void* stream) {
    if (!x || !w || !y || !gstat || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    DwmArgs a;
    if (!dwm_plan(a, B, C, H, W, K, pad)) return VFM_NO_KERNEL;
    if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)noise | (uintptr_t)gstat) % 16) return VFM_NO_KERNEL;
    a.x = (const __hip_bfloat16*)x; a.w = w; a.bias = bias; a.noise = noise; a.y = (__hip_bfloat16*)y;
    a.res = nullptr; a.nplane = nullptr; a.npart = nullptr; a.gstat = gstat; a.flip = 0;
    hipStream_t st = (hipStream_t)stream;
    switch (K) {
    case 3: return dwm_launch<3>(a, st);
    case 5: return dwm_launch<5>(a, st);
    default: return dwm_launch<7>(a, st);
    }
}

// entries of vfm_dwconv2d_fwd_mfma_nz's npart; VFM_NO_KERNEL if the shape is not covered
extern "C" long long vfm_dwconv2d_fwd_mfma_units(int B, int C, int H, int W, int K, int pad) {
    DwmArgs a;
    if (!dwm_plan(a, B, C, H, W, K, pad)) return VFM_NO_KERNEL;
    return a.units;
}

extern "C" int vfm_dwconv2d_fwd_mfma_ex(const void* x, const float* w, const float* bias, const float* noise,
                                        const void* res, void* y, int B, int C, int H, int W, int K, int pad, int flip,
                                        void* stream) {
    return vfm_dwconv2d_fwd_mfma_nz(x, w, bias, noise, res, y, nullptr, nullptr, B, C, H, W, K, pad, flip, stream);
}

extern "C" int vfm_dwconv2d_fwd_mfma(const void* x, const float* w, const float* bias, const float* noise,
                                     const void* res, void* y, int B, int C, int H, int W, int K, int pad,
                                     void* stream) {
    return vfm_dwconv2d_fwd_mfma_ex(x, w, bias, noise, res, y, B, C, H, W, K, pad, 0, stream);
}

// tiles (rows of the partial buffer) of vfm_dwconv2d_bwd_weight_mfma; VFM_NO_KERNEL if not covered
extern "C" int vfm_dwconv2d_bwd_weight_mfma_tiles(int B, int C, int H, int W, int K, int pad) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    if ((K != 3 && K != 5 && K != 7) || pad != (K - 1) / 2 || W % 16) return VFM_NO_KERNEL;
    DwmBwArgs a{};
    int XW;
    if (!dwm_bw_plan(a, B, C, H, W, XW)) return VFM_NO_KERNEL;
    return a.tiles;
}

// partial[t, c, :] (t < tiles): per-wave sums of dW[c] (K K taps) and db[c] over bf16 NCHW x / dy
extern "C" int vfm_dwconv2d_bwd_weight_mfma(const void* x, const void* dy, float* partial, int B, int C, int H, int W,
                                           int K, int pad, void* stream) {
    if (!x || !dy || !partial || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    if ((K != 3 && K != 5 && K != 7) || pad != (K - 1) / 2 || W % 16) return VFM_NO_KERNEL;
    if (((uintptr_t)x | (uintptr_t)dy) % 16) return VFM_NO_KERNEL;
    DwmBwArgs a{};
    int XW;
    if (!dwm_bw_plan(a, B, C, H, W, XW)) return VFM_NO_KERNEL;
    a.x = (const __hip_bfloat16*)x; a.dy = (const __hip_bfloat16*)dy; a.partial = partial;
    hipStream_t st = (hipStream_t)stream;
    switch (K) {
    case 3: return dwm_bw_launch<3>(a, XW, st);
    case 5: return dwm_bw_launch<5>(a, XW, st);
    default: return dwm_bw_launch<7>(a, XW, st);
    }
}
