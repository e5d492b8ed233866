// 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on the MFMA cores, fp32 products as the
// f32x6 bf16 split (fp32-equivalent; f32x3 opt-in) -- the LPIPS VGG16 stack: reference
// training/lpips.py:126-163, run in fp32 by the reference; MIOpen's fp32 Winograd was the single
// largest kernel of the training step.
//
//   out[p, n] = epi( sum_{tap, c} x[p + shift(tap), c] * w[n, tap, c] ),   p = (b, y, x) pixels,
//   epi: + bias[n], ReLU, and/or x (mask[p, n] > 0) (the ReLU derivative of the layer below, for
//   the data-gradient pass), fp32 out.
//
// Layout: activations NHWC fp32 ([B, H, W, C] contiguous: channels_last), weights pre-split into NP bf16
// piece arrays [NP][Cout][ldw] (rows padded to ldw), k ordered tap-major (k = tap Cin + c) for Cin < 32 and
// channel-chunk-major for Cin >= 32 (k = (c / 32) 288 + tap 32 + c % 32: a K-tile is one tap of one
// 32-channel chunk, and the 9 taps of a chunk are consecutive K-tiles -- StageA::load_wide). Cin is a power of two >= 4 (the 3-channel image is padded to 4), Cout a multiple
// of 64. The data gradient of the same conv is this kernel with the flipped, transposed weights
// w'[cin, tap, cout] = w[cout, 8 - tap, cin] over dZ.
//
// GEMM view: M = B*H*W pixels, N = Cout, K = 9*Cin (tap-major). Tile BM pixels x BN couts x 32 k with
// 2 BM threads as (BM/64) x 2 waves of 64 x BN/2, 32x32x16 bf16 MFMA: 256 x 128 with 8 waves (two per
// SIMD: one wave's MFMAs overlap the other's loads, split and LDS writes) for the f32x6 products at
// Cout % 128 == 0 (vggbench: 146 -> 196 TF/s; 256 x 64 measured no faster than 128 x 64 for the
// Cout = 64 layers), 128 x BN with 4 waves otherwise; fp32 activations split into NP piece images on
// the way into LDS, the Terms<NP> piece products accumulated (gemm.hip's f32x6 / f32x3: hi.hi in
// its own accumulator). Two LDS stages (double buffer): the split + store of K-tile t+1 and the
// global loads of K-tile t+2 are issued between the MFMA steps of K-tile t, one barrier per K-tile
// (raw s_barrier after lgkmcnt(0): the in-flight global loads are not drained). The A loader is
// implicit: each thread owns 4 pixel rows and one 4-channel column of the tile; a k-tile (32
// channels of one tap, or for Cin < 32 several taps) becomes one 16-B load per row at
// (p + dy*W + dx)*Cin + c, zero outside the image. The 9 shifted reads of a pixel hit L2.
#include "vfm_common.h"

#include <cstdlib>

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int ROWB = BK * 2;          // bytes of one bf16 image row (4 16-B chunks)

struct ConvArgs {
    const float* x;      // [B, H, W, Cin]
    const __hip_bfloat16* w;    // [NP][Cout, ldw] pieces of w (hi[, mid], lo), tap-major k, zero-padded to ldw
    int ldw;
    long long wps;              // elements between pieces (Cout * ldw)
    const float* bias;   // [Cout] or null
    const float* mask;   // [B, H, W, Cout] or null
    float* out;          // [B, H, W, Cout]
    int M, H, W, Cin, lc, Cout, K;
    FastDiv fW, fH;
    int relu;
};

// [rows][32 k] bf16 image, 64-B rows: 16-B chunk ch of row at chunk ch ^ ((row >> 2) & 3) -- the 16
// rows of each ds_read_b128 lane group (same chunk) land on 16 distinct 16-B slots of the 256-B
// bank row (MI355X_MICROARCH.md §LDS), and a ds_write_b64 / ds_write_b128 lane group covers two /
// one whole 128-B row pairs
__device__ __forceinline__ int k32_off(int row, int ch) { return row * ROWB + 16 * (ch ^ ((row >> 2) & 3)); }

// 4 fp32 (one uint4) -> the NP pieces' halves of a 16-B image chunk (piece p at img + p * pstride)
template <int NP>
__device__ __forceinline__ void put4(unsigned char* img, int pstride, int off, uint4 r) {
    uint32_t p01[NP], p23[NP];
    split_pieces<NP>(__uint_as_float(r.x), __uint_as_float(r.y), p01);
    split_pieces<NP>(__uint_as_float(r.z), __uint_as_float(r.w), p23);
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(img + p * pstride + off) = make_uint2(p01[p], p23[p]);
}

// thread -> (row = tid/8 + (THREADS/8) u, 4-element column tid%8) of a [4 THREADS/8][32] fp32 tile
template <int THREADS>
struct StageA {
    static constexpr int IMG = 4 * (THREADS / 8) * ROWB;   // bytes of one bf16 piece image of the A tile
    uint4 r[4];
    int pm[4];    // pixel index (or -1)
    int pyx[4];   // y << 16 | x
    __device__ __forceinline__ void init(const ConvArgs& a, int m0, int tid) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int m = m0 + tid / 8 + (THREADS / 8) * u;
            if (m < a.M) {
                const uint32_t q = fdiv((uint32_t)m, a.fW);
                const int xx = m - (int)q * a.W;
                const int yy = (int)q - (int)fdiv(q, a.fH) * a.H;
                pm[u] = m;
                pyx[u] = (yy << 16) | xx;
            } else {
                pm[u] = -1;
                pyx[u] = 0;
            }
        }
    }
    // Cin < 32 (the 4-channel image layer): the taps of a K-tile differ per column
    __device__ __forceinline__ void load(const ConvArgs& a, int k0, int tid) {
        const int k = k0 + 4 * (tid & 7);
        const int tap = k >> a.lc, c = k & (a.Cin - 1);
        const int dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
        const bool tap_ok = tap < 9;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int yy = (pyx[u] >> 16) + dy, xx = (pyx[u] & 0xffff) + dx;
            const bool ok = tap_ok && pm[u] >= 0 && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
            r[u] = ok ? *reinterpret_cast<const uint4*>(a.x + (long long)(pm[u] + dy * a.W + dx) * a.Cin + c)
                      : make_uint4(0, 0, 0, 0);
        }
    }
    // Cin >= 32: a K-tile is 32 channels of ONE tap, so the 4 rows' validity and 32-bit element offsets
    // (pixel + tap shift, times Cin) change only with the tap; per K-tile only the channel offset moves
    int off[4];
    unsigned okm;
    int cur_tap;
    __device__ __forceinline__ void tap_setup(const ConvArgs& a, int tap) {
        const int dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
        okm = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int yy = (pyx[u] >> 16) + dy, xx = (pyx[u] & 0xffff) + dx;
            const bool ok = pm[u] >= 0 && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
            okm |= (unsigned)ok << u;
            off[u] = ok ? (pm[u] + dy * a.W + dx) * a.Cin : 0;
        }
        cur_tap = tap;
    }
    // K order for Cin >= 32 is channel-chunk-major, tap-minor: K-tile kt = 32 channels (kt / 9) x tap kt % 9,
    // so the 9 shifted reads of a pixel's channel chunk are 9 consecutive K-tiles and hit L2 (tap-major
    // order re-read them Cin / 32 K-tiles apart, from HBM: 3.75x the algorithmic traffic in round 3)
    __device__ __forceinline__ void load_wide(const ConvArgs& a, int k0, int tid) {
        const int kt = k0 >> 5;                          // uniform
        const int cc = kt / 9, tap = kt - 9 * cc;
        if (tap != cur_tap) tap_setup(a, tap);
        const int c = 32 * cc + 4 * (tid & 7);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            r[u] = ((okm >> u) & 1)
                       ? *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.x) + (unsigned)(off[u] + c) * 4u)
                       : make_uint4(0, 0, 0, 0);
    }
    template <int NP>
    __device__ __forceinline__ void store(unsigned char* img, int tid) const {
        const int cc = tid & 7;
#pragma unroll
        for (int u = 0; u < 4; ++u) put4<NP>(img, IMG, k32_off(tid / 8 + (THREADS / 8) * u, cc >> 1) + 8 * (cc & 1), r[u]);
    }
};

// weights arrive pre-split (NP bf16 pieces, split once per weight version on the host side):
// thread -> 16-B chunks (8 k) c = tid + THREADS u of a [ROWS][32] tile, copied as-is into the piece
// images (with more threads than chunks, the threads past ROWS * 4 load nothing)
template <int ROWS, int NP, int THREADS>
struct StageB {
    static constexpr int CHUNKS = ROWS * 4;
    static constexpr int PER = CHUNKS >= THREADS ? CHUNKS / THREADS : 1;
    static constexpr int IMG = ROWS * ROWB;
    uint4 v[NP][PER];
    __device__ __forceinline__ void load(const ConvArgs& a, int n0, int k0, int tid) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int c = tid + THREADS * u, row = c >> 2, k = k0 + 8 * (c & 3), n = n0 + row;
            const bool ok = k < a.ldw && n < a.Cout && c < CHUNKS;
            const unsigned o = (unsigned)(n * a.ldw + k) * 2u;          // byte offset (host: Cout * ldw < 2^30)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                v[p][u] = ok ? *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.w + p * a.wps) + o)
                             : make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void store(unsigned char* img, int tid) const {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int c = tid + THREADS * u, off = k32_off(c >> 2, c & 3);
            if (CHUNKS < THREADS && c >= CHUNKS) continue;
#pragma unroll
            for (int p = 0; p < NP; ++p) *reinterpret_cast<uint4*>(img + p * IMG + off) = v[p][u];
        }
    }
};

// MFMA operand fragment: 32-row block blk, k16 step s: lane (r, hh) holds row 32 blk + r, k = 16 s + 8 hh .. +7
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int blk, int s, int lane) {
    return *reinterpret_cast<const bf16x8*>(img + k32_off(32 * blk + (lane & 31), 2 * s + (lane >> 5)));
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// BM x BN tile, THREADS = 2 BM: waves as (BM / 64) (M) x 2 (N), each 64 rows x BN / 2 columns.
template <int BM, int BN, int NP>
__global__ __launch_bounds__(2 * BM, (BM == 256 || (NP == 3 && BN == 128)) ? 1 : 2) void conv3x3_kernel(ConvArgs a) {
    constexpr int THREADS = 2 * BM;
    constexpr int WM = BM / 64;                 // waves along M
    constexpr int NJ = BN / 64;                 // 32-col blocks per wave
    constexpr int IMG_A = StageA<THREADS>::IMG;
    constexpr int IMG_B = BN * ROWB;
    constexpr int STAGE = NP * (IMG_A + IMG_B); // A pieces, then B pieces
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave % WM, wn = wave / WM;
    const int tiles_n = a.Cout / BN;
    // XCD-aware bijective remap: the blocks b, b+8, b+16, ... (one XCD, one L2) take consecutive
    // tiles, i.e. all Cout tiles of neighbouring pixel rows, which share the same input rows
    // (9 taps x Cout/BN reads of every input pixel then hit that XCD's L2)
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;

    StageA<THREADS> sa;
    StageB<BN, NP, THREADS> sb;
    sa.init(a, m0, tid);
    sa.cur_tap = -1;
    const bool wide = a.lc >= 5;                        // Cin >= 32 (uniform)
    f32x16 acc[2][NJ], accs[2][NJ];             // hi.hi products / the smaller piece products
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = accs[i][j] = f32x16{};

    const int KT = (a.K + BK - 1) / BK;
    auto gload = [&](int kt) {
        if (wide) sa.load_wide(a, kt * BK, tid);
        else sa.load(a, kt * BK, tid);
        sb.load(a, n0, kt * BK, tid);
    };
    auto lstore = [&](int buf) {
        unsigned char* st = lds + buf * STAGE;
        sa.template store<NP>(st, tid);
        sb.store(st + NP * IMG_A, tid);
    };
    gload(0);
    lstore(0);
    if (KT > 1) gload(1);
    lds_barrier();
    for (int kt = 0; kt < KT; ++kt) {
        const unsigned char* ca = lds + (kt & 1) * STAGE;
        const unsigned char* cb = ca + NP * IMG_A;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 af[NP][2], bf[NP][NJ];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
#pragma unroll
                for (int i = 0; i < 2; ++i) af[p][i] = frag(ca + p * IMG_A, 2 * wm + i, s, lane);
#pragma unroll
                for (int j = 0; j < NJ; ++j) bf[p][j] = frag(cb + p * IMG_B, NJ * wn + j, s, lane);
            }
            // small piece products into their own accumulator (rounded at their own ~2^-8 scale),
            // hi.hi alone into acc: as many full-magnitude roundings as an fp32 GEMM of exact products
#pragma unroll
            for (int t = 0; t < Terms<NP>::N; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        f32x16& c = (t == Terms<NP>::N - 1) ? acc[i][j] : accs[i][j];
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[Terms<NP>::a(t)][i], bf[Terms<NP>::b(t)][j], c,
                                                                    0, 0, 0);
                    }
            // between the two MFMA steps: K-tile kt+1 from registers into the other stage, then the
            // global loads of K-tile kt+2 (its stage was last read before the previous barrier)
            if (s == 0 && kt + 1 < KT) {
                lstore((kt + 1) & 1);
                if (kt + 2 < KT) gload(kt + 2);
            }
        }
        lds_barrier();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] += accs[i][j];

    // acc[i][j][e] = out[m][n], m = m0 + 64wm + 32i + (e&3) + 8(e>>2) + 4hh, n = n0 + 32(NJ wn + j) + r
    const int r = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = n0 + 32 * (NJ * wn + j) + r;
        const float bn = a.bias ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + 64 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
                if (m >= a.M) continue;
                const unsigned o = (unsigned)(m * a.Cout + n) * 4u;     // byte offset (host: M * Cout < 2^30)
                float v = acc[i][j][e] + bn;
                if (a.relu) v = fmaxf(v, 0.f);
                if (a.mask && !(*reinterpret_cast<const float*>(reinterpret_cast<const char*>(a.mask) + o) > 0.f)) v = 0.f;
                *reinterpret_cast<float*>(reinterpret_cast<char*>(a.out) + o) = v;
            }
    }
}

template <int BM, int BN, int NP>
int launch(const ConvArgs& a, hipStream_t st) {
    const size_t lds = 2 * NP * (BM + BN) * ROWB;
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)conv3x3_kernel<BM, BN, NP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr[dv_attr] = true;
    }
    const long long tiles = (long long)((a.M + BM - 1) / BM) * (a.Cout / BN);
    if (tiles > 0x7fffffff) return VFM_ERR_ARGS;
    VFM_LAUNCH((conv3x3_kernel<BM, BN, NP>), dim3((unsigned)tiles), dim3(2 * BM), lds, st, a);
    return launch_status();
}

}  // namespace

extern "C" int vfm_conv3x3_nhwc_f32(const float* x, const void* w_pieces, int precision, int ldw, const float* bias,
                                    const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int relu,
                                    void* stream) {
    if (!x || !w_pieces || !out || B <= 0 || H <= 0 || W <= 0 || H > 32767 || W > 32767) return VFM_ERR_ARGS;
    if (precision != VFM_F32 && precision != VFM_F32X3) return VFM_ERR_ARGS;
    const int np = precision == VFM_F32 ? 3 : 2;
    if (Cin < 4 || (Cin & (Cin - 1)) || Cout <= 0 || Cout % 64) return VFM_NO_KERNEL;
    if (ldw < 9 * Cin || ldw % 64) return VFM_ERR_ARGS;
    if (((uintptr_t)x | (uintptr_t)w_pieces) % 16) return VFM_ERR_ARGS;
    const long long M = (long long)B * H * W;
    if (M * (long long)(Cin > Cout ? Cin : Cout) >= (1ll << 40) || M >= (1ll << 31) - 2 * (long long)W - 2)
        return VFM_ERR_ARGS;
    // 32-bit byte offsets in the loaders / epilogue
    if (Cin >= 64 && (M + 2 * (long long)W + 2) * Cin >= (1ll << 30)) return VFM_ERR_ARGS;
    if (M * (long long)Cout >= (1ll << 30) || (long long)Cout * ldw >= (1ll << 30)) return VFM_ERR_ARGS;
    ConvArgs a;
    a.x = x; a.w = (const __hip_bfloat16*)w_pieces; a.ldw = ldw; a.wps = (long long)Cout * ldw;
    a.bias = bias; a.mask = mask; a.out = out;
    a.M = (int)M; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.K = 9 * Cin;
    a.lc = 0;
    while ((1 << a.lc) < Cin) ++a.lc;
    a.fW = make_fastdiv((uint32_t)W);
    a.fH = make_fastdiv((uint32_t)H);
    a.relu = relu;
    hipStream_t st = (hipStream_t)stream;
    // Cout = 64 layers (conv1_x): 128 x 64 tiles with 4 waves, two workgroups per CU; VFM_CONV_N64=256 runs
    // them on 256 x 64 tiles with 8 waves (A/B: 3.10 vs 2.96 ms for the 64-image forward,
    // profiles/r4_q_conv_n64_ab.txt -- the larger tile does not pay)
    static const bool wide64 = [] {
        const char* e = getenv("VFM_CONV_N64");
        return e && e[0] == '2';
    }();
    if (np == 3) {
        if (Cout % 128 == 0) return launch<256, 128, 3>(a, st);
        return wide64 ? launch<256, 64, 3>(a, st) : launch<128, 64, 3>(a, st);
    }
    return (Cout % 128 == 0) ? launch<128, 128, 2>(a, st) : launch<128, 64, 2>(a, st);
}

// ---------------------------------------------------------------------------------------------
// Input gradient of the image layer (3 -> 64 channels) of the VGG16 stack: few output channels, so
// neither the implicit GEMM above (Cout % 64) nor MFMA fits; exact fp32 FMAs on the VALU
// (replaces the MIOpen fp32 Winograd that torch.nn.grad.conv2d_input ran here).
//   dx[b, c, y, x] = sum_{o, ky, kx} w[o, c, ky, kx] dz[b, y + 1 - ky, x + 1 - kx, o]   (zero outside)
// dz NHWC fp32 [B, H, W, K] (K % 4 == 0, K <= 128), w fp32 [K][C][3][3] (the forward weight, torch
// layout), dx NCHW fp32 [B, C, H, W], C <= 4. A workgroup = 64 pixels of one image row x 4 channel
// groups: the 3 input rows x 66 pixels it touches are staged in LDS once (coalesced 16-B loads, pixel
// stride K + 4 floats so the 16 lanes of a ds_read_b128 group hit 16 different bank slots), each
// thread sums K / 4 channels of its pixel for all C outputs, and the 4 partial sums per pixel are
// combined with two xor-shuffles in a fixed order (deterministic).
namespace {

constexpr int DG_PX = 64;

template <int C>
__global__ __launch_bounds__(256) void conv3x3_dgrad_small(const float* __restrict__ dz, const float* __restrict__ w,
                                                           float* __restrict__ dx, int H, int W, int K) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int KP = K + 4;                                   // padded pixel stride (floats)
    float* tile = sm;                                       // [3][DG_PX + 2][KP]
    float* ws = sm + 3 * (DG_PX + 2) * KP;                  // [9][C][K]: ws[(tap * C + c) * K + o]
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * DG_PX, y = blockIdx.y, b = blockIdx.z;
    for (int i = tid; i < 9 * C * K; i += 256) {
        const int o = i % K, c = (i / K) % C, tap = i / (K * C);
        ws[i] = w[((long long)o * C + c) * 9 + tap];
    }
    const int K4 = K >> 2;
    for (int i = tid; i < 3 * (DG_PX + 2) * K4; i += 256) {
        const int q = i % K4, px = (i / K4) % (DG_PX + 2), r = i / (K4 * (DG_PX + 2));
        const int yy = y + 1 - r, xx = x0 - 1 + px;        // row r holds dz row y + 1 - r (ky = r)
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
            v = *reinterpret_cast<const float4*>(dz + (((long long)b * H + yy) * W + xx) * K + 4 * q);
        *reinterpret_cast<float4*>(tile + (r * (DG_PX + 2) + px) * KP + 4 * q) = v;
    }
    __syncthreads();
    const int px = tid & (DG_PX - 1), cg = tid >> 6;        // pixel, channel group (K / 4 channels each)
    const int kq = K >> 2, kb = cg * kq;
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            // x' + 1 - kx = x0 + px + 1 - kx  ->  staged column px + 2 - kx
            const float* src = tile + (ky * (DG_PX + 2) + px + 2 - kx) * KP + kb;
            const float* wt = ws + (ky * 3 + kx) * C * K + kb;
            for (int o = 0; o < kq; o += 4) {
                const float4 d = *reinterpret_cast<const float4*>(src + o);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const float4 wv = *reinterpret_cast<const float4*>(wt + c * K + o);
                    acc[c] = fmaf(d.x, wv.x, acc[c]);
                    acc[c] = fmaf(d.y, wv.y, acc[c]);
                    acc[c] = fmaf(d.z, wv.z, acc[c]);
                    acc[c] = fmaf(d.w, wv.w, acc[c]);
                }
            }
        }
    // combine the 4 channel groups (lanes px, px+64, ... live in different waves): through LDS
    __syncthreads();
    float* red = sm;                                        // [4][C][DG_PX]
#pragma unroll
    for (int c = 0; c < C; ++c) red[(cg * C + c) * DG_PX + px] = acc[c];
    __syncthreads();
    if (tid < DG_PX * C) {
        const int p = tid % DG_PX, c = tid / DG_PX, xx = x0 + p;
        const float v = ((red[(0 * C + c) * DG_PX + p] + red[(1 * C + c) * DG_PX + p]) + red[(2 * C + c) * DG_PX + p]) +
                        red[(3 * C + c) * DG_PX + p];
        if (xx < W) dx[(((long long)b * C + c) * H + y) * W + xx] = v;
    }
}

template <int C>
int launch_dgrad(const float* dz, const float* w, float* dx, int B, int H, int W, int K, hipStream_t st) {
    const size_t lds = (3 * (DG_PX + 2) * (size_t)(K + 4) + 9 * (size_t)C * K) * 4;
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)conv3x3_dgrad_small<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (3 * (DG_PX + 2) * (128 + 4) + 9 * 4 * 128) * 4);
        attr[dv_attr] = true;
    }
    VFM_LAUNCH((conv3x3_dgrad_small<C>), dim3((W + DG_PX - 1) / DG_PX, H, B), dim3(256), lds, st, dz, w, dx, H, W,
                       K);
    return launch_status();
}

}  // namespace

extern "C" int vfm_conv3x3_dgrad_small_f32(const float* dz, const float* w, float* dx, int B, int H, int W, int C,
                                           int K, void* stream) {
    if (!dz || !w || !dx || B <= 0 || H <= 0 || W <= 0 || B > 65535 || H > 65535) return VFM_ERR_ARGS;
    if (C < 1 || C > 4 || K % 4 || K <= 0 || K > 128 || ((uintptr_t)dz % 16)) return VFM_NO_KERNEL;
    hipStream_t st = (hipStream_t)stream;
    switch (C) {
    case 1: return launch_dgrad<1>(dz, w, dx, B, H, W, K, st);
    case 2: return launch_dgrad<2>(dz, w, dx, B, H, W, K, st);
    case 3: return launch_dgrad<3>(dz, w, dx, B, H, W, K, st);
    default: return launch_dgrad<4>(dz, w, dx, B, H, W, K, st);
    }
}
