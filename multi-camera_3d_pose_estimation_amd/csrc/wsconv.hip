// Weight-stationary 3x3/s1 convolutions for the HRNet branch BasicBlocks (gfx950).
//
// The branch convs with Cin = Cout = C on a fixed plane (64 ch at 32x24, 128 ch
// at 16x12; 120 of HRNet-W32's 293 convs) are, per crop, a small GEMM
// (M = C couts, N = H*W pixels, K = 9C) repeated over ~1000 crops.  Here each
// wave keeps its share of the BN-folded weights in VGPRs for the whole launch
// (64 couts x 576 k = 72 A fragments = 288 VGPRs, one wave per SIMD), so a B
// (pixel) fragment read from LDS feeds 4 MFMAs (v_mfma_f32_16x16x32_bf16) and
// LDS runs at ~25 % of its bandwidth.  Per tile (TH rows of one crop) the only
// traffic is the input halo — LDS-DMA (global_load_lds) into a double buffer,
// one barrier per tile, the next tile's halo streaming under this tile's
// MFMAs — plus the residual and the output.  LDS images are NHWC with the
// 16-B channel chunks of a pixel XOR-swizzled by pixel index (source-side
// permutation, linear DMA destination), so the 16-lane groups of a fragment
// read spread over the bank row.  C = 128 (295 KB of weights) splits K over
// wave pairs: the second wave of a pair hands its partial sums to the first
// through LDS (one barrier per round).
// Since the pixel-major tconv halo, the 128-ch plane runs tconv_kernel by default; this
// kernel serves it with MVPOSE_TCONV128=0 (and the 64-ch plane with MVPOSE_WSCONV64=1).
// K order is (tap, cin); conv_mfma_kernel sums the same products in (cin chunk,
// tap) order, so the two agree to f32 rounding, not bit for bit.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mvp_common.h"

namespace mvp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float relu(float v) {  // one v_max_f32 (fmaxf adds a canonicalize)
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {  // RNE, one v_cvt_pk_bf16_f32
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

template <int C, int H, int W, int TH>
struct WsCfg {
    static constexpr int NW = 4, NT = 256;
    static constexpr int KSPLIT = C >= 128 ? 2 : 1;
    static constexpr int NCG = C / 64;                    // 64-cout groups
    static constexpr int CTW = 4;                         // 16-cout tiles per wave
    static constexpr int KPT = C / 32;                    // 32-deep k-steps per tap
    static constexpr int KSW = 9 * KPT / KSPLIT;          // k-steps per wave
    static constexpr int NPG = NW / (NCG * KSPLIT);       // pixel groups
    static constexpr int HH = TH + 2, HW = W + 2, HPIX = HH * HW;
    static constexpr int PB = 2 * C;                      // bytes per NHWC pixel
    static constexpr int CH = C / 8;                      // 16-B chunks per pixel
    static constexpr int PPR = PB >= 256 ? 1 : 256 / PB;  // pixels per 256-B bank row
    static constexpr int PIECES = (HPIX * PB + NT * 16 - 1) / (NT * 16);  // 1-KiB DMA pieces per wave
    static constexpr int HBYTES = PIECES * NT * 16;
    static constexpr int OPIX = TH * W, PT = OPIX / 16, PTW = PT / NPG;
    static constexpr int RP = 2, ROUNDS = PTW / RP;       // pixel tiles per round, rounds per tile
    static constexpr int PART = RP * CTW * 64 * 16;       // one wave's partial sums of one round
    static constexpr int PART_OFF = 2 * HBYTES;
    static constexpr int BIAS_OFF = PART_OFF + (KSPLIT == 2 ? 2 * NCG * PART : 0);
    static constexpr int LDS = BIAS_OFF + C * 4;
    static constexpr int EPI_STORES = PTW * CTW;          // stores per epilogue wave per tile
    static_assert(C % 64 == 0 && H % TH == 0 && OPIX % 16 == 0 && PT % NPG == 0 && PTW % RP == 0, "tiling");
    static_assert(NCG * KSPLIT * NPG == NW, "wave roles");
    static_assert(EPI_STORES < 64, "vmcnt is 6 bits");
    static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct WsParams {
    const uint16_t* x;
    const uint16_t* w;
    const float* bias;
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* zero;
    int n_tiles;
};

template <int C, int H, int W, int TH, bool RES>
__global__ __launch_bounds__(256, 1) void wsconv_kernel(WsParams p) {
    using G = WsCfg<C, H, W, TH>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cg = wave % G::NCG;
    const int kh = (wave / G::NCG) % G::KSPLIT;
    const int pg = wave / (G::NCG * G::KSPLIT);
    const bool epi = kh == 0;  // the wave that finishes (bias, residual, ReLU, store) its cout group
    const int co_w = cg * 64;
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = H / TH;
    float* sbias = reinterpret_cast<float*>(lds + G::BIAS_OFF);
    if (tid < C) sbias[tid] = p.bias[tid];  // visible after the first tile's barrier

    // ---- this wave's weights, resident for the launch: A fragment [ct][s] =
    // couts co_w + 16ct .. +15 x k-step kh*KSW + s (k = tap*C + cin, 8 k per lane)
    bf16x8 wf[G::CTW][G::KSW];
    {
        const uint16_t* wl = p.w + (size_t)(co_w + (lane & 15)) * 9 * C + kh * G::KSW * 32 + (lane >> 4) * 8;
#pragma unroll
        for (int ct = 0; ct < G::CTW; ct++)
#pragma unroll
            for (int s = 0; s < G::KSW; s++)
                wf[ct][s] = *reinterpret_cast<const bf16x8*>(wl + (size_t)ct * 16 * 9 * C + s * 32);
    }

    // ---- per-lane halo geometry of this wave's DMA pieces (fixed for the launch).
    // LDS byte o holds chunk slot (o % PB)/16 of halo pixel o / PB; the chunk stored
    // there is slot ^ swz(pixel), so the global source address carries the swizzle.
    // packed per piece: halo row | halo col << 5 | source chunk << 10 (-1: past the halo)
    int hgeo[G::PIECES];
#pragma unroll
    for (int j = 0; j < G::PIECES; j++) {
        const int o = (j * G::NW + wave) * 1024 + lane * 16;
        const int hp = o / G::PB, slot = (o % G::PB) / 16;
        const int q = slot ^ ((hp / G::PPR) & (G::CH - 1));
        const int hr = hp / G::HW, hc = hp - (hp / G::HW) * G::HW;
        hgeo[j] = hp < G::HPIX ? (hr | (hc << 5) | (q << 10)) : -1;
    }
    auto issue = [&](int k, uint8_t* hb) {
        const int tile = blockIdx.x + k * gridDim.x;
        const bool tile_ok = tile < p.n_tiles;
        const int n = tile / tiles_h, ho0 = (tile - (tile / tiles_h) * tiles_h) * TH;
        const uint16_t* xb = p.x + (((long)n * H + ho0 - 1) * W - 1) * C;
#pragma unroll
        for (int j = 0; j < G::PIECES; j++) {
            const int g = hgeo[j];
            const int hr = g & 31, hc = (g >> 5) & 31, q = g >> 10;
            const bool in = tile_ok && g >= 0 && (unsigned)(ho0 - 1 + hr) < (unsigned)H && (unsigned)(hc - 1) < (unsigned)W;
            // out-of-image slots read a distinct 16-B slot of the zero region per lane
            const void* src = in ? (const void*)(xb + (hr * W + hc) * C + q * 8)
                                 : (const void*)(p.zero + (((j * G::NW + wave) * 64 + lane) & 4095) * 8);
            glds16(src, hb + (j * G::NW + wave) * 1024);
        }
    };

    // ---- B fragments: lane reads pixel (lane & 15) of a 16-pixel tile, chunk (lane >> 4) of a k-step.
    // Byte address of (halo pixel hp, chunk q) = hp*PB + (q ^ swz(hp))*16 with swz < CH, so for one
    // tap the k-steps of that tap differ only by an XOR of (kq*4)*16 on the tap's kq=0 address.
    const int l4 = lane >> 4;
    auto tap_addr = [&](int hp0, int tap, int buf_off) -> int {
        const int hp = hp0 + (tap / 3) * G::HW + tap % 3;
        const int sw = ((unsigned)hp / G::PPR) & (G::CH - 1);
        return buf_off + hp * G::PB + ((l4 ^ sw) << 4);
    };
    auto pix_base = [&](int t) -> int {  // halo pixel of output pixel tile t's lane pixel, tap (0,0)
        unsigned ipx = (pg * G::PTW + t) * 16 + (lane & 15);
        asm volatile("" : "+v"(ipx));  // recomputed per round: keeps PTW x 9 addresses from being hoisted
        return (int)((ipx / W) * G::HW + ipx % W);
    };

    const int n_items = (p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    issue(0, lds);
    for (int k = 0; k < n_items; k++) {
        const int buf_off = (k & 1) * G::HBYTES;
        // this wave's pieces of tile k have landed (the only younger vector-memory ops
        // are the previous tile's stores); the barrier publishes every wave's pieces and
        // retires all reads of the other buffer, which the next DMA overwrites
        if (k == 0 || !epi)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::EPI_STORES) : "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, ho0 = (tile - (tile / tiles_h) * tiles_h) * TH;
        const long pix0 = ((long)n * H + ho0) * W;
        // residual rows of the whole tile, issued BEFORE the next halo's DMA so that
        // waiting for them never waits for it
        uint2 rv[G::PTW][G::CTW];
        if constexpr (RES) {
            if (epi) {
#pragma unroll
                for (int t = 0; t < G::PTW; t++)
#pragma unroll
                    for (int ct = 0; ct < G::CTW; ct++)
                        rv[t][ct] = *reinterpret_cast<const uint2*>(
                            p.res + (pix0 + (pg * G::PTW + t) * 16 + (lane & 15)) * C + co_w + ct * 16 + l4 * 4);
            }
        }
        asm volatile("" ::: "memory");
        issue(k + 1, lds + ((k + 1) & 1) * G::HBYTES);  // past the end: zero reads into the free buffer
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < G::ROUNDS; r++) {
            // accumulators start at the folded-BN bias (the K-half-1 wave of a split starts at 0)
            f32x4 acc[G::RP][G::CTW];
#pragma unroll
            for (int ct = 0; ct < G::CTW; ct++) {
                const f32x4 bb = epi ? *reinterpret_cast<const f32x4*>(sbias + co_w + ct * 16 + l4 * 4)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < G::RP; i++) acc[i][ct] = bb;
            }
            int hpb[G::RP];
#pragma unroll
            for (int i = 0; i < G::RP; i++) hpb[i] = pix_base(r * G::RP + i);
            const int gs0 = kh * G::KSW;
            int ta[G::RP];
            auto bread = [&](int i, int gs) -> bf16x8 {
                const int kq = gs % G::KPT;
                if (kq == 0 || gs == gs0) ta[i] = tap_addr(hpb[i], gs / G::KPT, buf_off);
                return *reinterpret_cast<const bf16x8*>(lds + (ta[i] ^ (kq * 64)));
            };
            // fragments of k-step s+1 are read before the MFMAs of step s (two register sets)
            bf16x8 fb[2][G::RP];
#pragma unroll
            for (int i = 0; i < G::RP; i++) fb[0][i] = bread(i, gs0);
#pragma unroll
            for (int s = 0; s < G::KSW; s++) {
                const int cur = s & 1;
                if (s + 1 < G::KSW) {
#pragma unroll
                    for (int i = 0; i < G::RP; i++) fb[cur ^ 1][i] = bread(i, gs0 + s + 1);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < G::RP; i++)
#pragma unroll
                    for (int ct = 0; ct < G::CTW; ct++)
                        acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][s], fb[cur][i], acc[i][ct], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (G::KSPLIT == 2) {
                // the K-half-1 wave of each cout group hands its partial sums to the K-half-0 wave
                f32x4* part = reinterpret_cast<f32x4*>(lds + G::PART_OFF + ((r & 1) * G::NCG + cg) * G::PART);
                if (!epi) {
#pragma unroll
                    for (int i = 0; i < G::RP; i++)
#pragma unroll
                        for (int ct = 0; ct < G::CTW; ct++) part[(i * G::CTW + ct) * 64 + lane] = acc[i][ct];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                if (epi) {
#pragma unroll
                    for (int i = 0; i < G::RP; i++)
#pragma unroll
                        for (int ct = 0; ct < G::CTW; ct++) acc[i][ct] += part[(i * G::CTW + ct) * 64 + lane];
                }
            }
            if (epi) {
                // [+ residual] + ReLU -> bf16 NHWC
#pragma unroll
                for (int i = 0; i < G::RP; i++) {
                    const int t = r * G::RP + i;
                    uint16_t* yrow = p.y + (pix0 + (pg * G::PTW + t) * 16 + (lane & 15)) * C + co_w + l4 * 4;
#pragma unroll
                    for (int ct = 0; ct < G::CTW; ct++) {
                        f32x4 v = acc[i][ct];
                        if constexpr (RES) {
                            const uint2 rr = rv[t][ct];
                            v[0] += __uint_as_float(rr.x << 16);
                            v[1] += __uint_as_float(rr.x & 0xffff0000u);
                            v[2] += __uint_as_float(rr.y << 16);
                            v[3] += __uint_as_float(rr.y & 0xffff0000u);
                        }
                        uint2 o;
                        o.x = pack_bf16x2(relu(v[0]), relu(v[1]));
                        o.y = pack_bf16x2(relu(v[2]), relu(v[3]));
                        *reinterpret_cast<uint2*>(yrow + ct * 16) = o;
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (zero) DMA has landed before the wave exits
}

int g_ws_cus = 0;

template <int C, int H, int W, int TH, bool RES>
void launch_ws_kernel(const WsParams& p, hipStream_t s) {
    using G = WsCfg<C, H, W, TH>;
    auto kern = wsconv_kernel<C, H, W, TH, RES>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (g_ws_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_ws_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int grid = std::min(p.n_tiles, g_ws_cus);  // one workgroup per CU (VGPRs: one wave per SIMD)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), G::LDS, s, p);
}

template <int C, int H, int W, int TH>
void launch_ws(const ConvLaunch& c, hipStream_t s) {
    const long tiles = (long)c.N * (H / TH);
    MVP_REQUIRE(tiles < (1L << 30), "wsconv: too many tiles");
    WsParams p{c.x, c.w, c.bias, c.res, c.y, conv_zero_region(), (int)tiles};
    if (c.res)
        launch_ws_kernel<C, H, W, TH, true>(p, s);
    else
        launch_ws_kernel<C, H, W, TH, false>(p, s);
}

}  // namespace

bool launch_wsconv(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 3 || c.stride != 1 || c.out_f32_nchw || c.Cin != c.Cout || !c.relu) return false;
    const char* e = getenv("MVPOSE_NO_WSCONV");  // diagnostics/tests: use the generic conv kernel
    if (e && e[0] == '1') return false;
    // 64 ch @ 32x24 compiles (and is tested) but measured slower than conv_mfma_kernel
    // (93.8 vs 111.5 us/conv at 1024 crops: residual prefetch spills); opt in with MVPOSE_WSCONV64=1
    const char* e64 = getenv("MVPOSE_WSCONV64");
    if (c.Cin == 64 && c.H == 32 && c.W == 24 && e64 && e64[0] == '1') {
        launch_ws<64, 32, 24, 16>(c, s);
        return true;
    }
    if (c.Cin == 128 && c.H == 16 && c.W == 12) {
        launch_ws<128, 16, 12, 8>(c, s);
        return true;
    }
    return false;
}

}  // namespace mvp
