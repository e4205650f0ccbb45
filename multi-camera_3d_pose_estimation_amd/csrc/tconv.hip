// Lean 3x3/s1 implicit-GEMM convolution on v_mfma_f32_32x32x16_bf16 (gfx950).
//
// Used for the stride-1 3x3 convs whose output tile is 384 pixels x 64 couts:
// the HRNet-W32 branch planes 64 ch @ 32x24 (whole rows), 256 ch @ 8x6 (8 crops
// per tile) and layer1's 64 ch @ 64x48.  The generic conv_mfma_kernel issues
// ~4.7 VALU instructions per 16x16x32 MFMA (64-bit address math, per-item
// bookkeeping; rocprofv3 SQ counters, profiles/), which caps it near 25 % of the
// MFMA peak.  This kernel is built so that the steady state issues almost
// nothing but MFMAs and LDS reads:
//
//  * 32x32x16 MFMAs (32 cycles each): twice the VALU issue slack per instruction
//    of 16x16x32 and half the instruction count.
//  * Every fragment read is ds_read_b128 [base VGPR + compile-time immediate]:
//    the halo is stored chunk-major ([8-channel group q][slot], 16-B slots) with a
//    row pitch of W+1 slots whose extra slot is zero, plus one leading zero slot.
//    A tap (dy, dx) of output pixel (y, x) is then slot base(y, x) + dy*(W+1) + dx
//    for EVERY pixel: the left/right image border reads a pad slot, so no lane
//    masking and no per-tap address math.  Weights sit in LDS as [tap][q][cout].
//  * One work item = (tile, 32-input-channel chunk); an item is 54 MFMAs per wave.
//    Its halo (and weight slice, unless the weights are LDS-resident) arrives by
//    LDS-DMA (global_load_lds) into the other half of a two-slot ring while the
//    current item computes; per-lane DMA geometry is precomputed once per launch.
//  * Weights of Cin = 64 convs (73.7 KiB) stay resident in LDS for the launch:
//    re-streaming them per item was 56 % of the DMA bytes (measured: no-DMA
//    diagnostic 46.5 us vs 109 us per conv at 1024 crops).
//  * Accumulator rows are a permutation of the couts (A row 8j+4h+i holds cout
//    16h+4j+i), so each lane owns 16 consecutive couts of its pixel: residual
//    loads and output stores are 2 x 16 B per lane and fragment instead of 4 x 8 B
//    (the store tail is issue-bound, MI355X_MICROARCH.md).
//  * Epilogue fused: accumulators start at the folded-BN bias; + residual, ReLU,
//    bf16 pack.
// 8 waves (2 per SIMD) per workgroup, one workgroup per CU, persistent over tiles.
// K order is (cin chunk, tap, cin within chunk); results agree with the other conv
// kernels to f32 summation-order rounding, not bit for bit.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;  // 16-B slots of the shared zero region


template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM_ = 64, bool PM_ = false>
struct TCfg {
    static constexpr int NW = 8, NT_THREADS = NW * 64;
    static constexpr int BM = BM_, MG = BM / 32, PG = NW / MG;  // cout groups x pixel groups
    static constexpr int NT = 3;                                 // 32-pixel fragments per wave
    static constexpr int P = NB * TH * W;                        // output pixels per tile
    static constexpr int NCH = CIN / 32;                         // items per tile
    // BLK: fragments are 8x4 pixel blocks (frag_pixel_blk) on a row pitch of W + 2 slots (= 2
    // mod 4): conflict-free B reads where 32-pixel raster fragments wrap rows (W = 12: the
    // raster map measured 43 % of the LDS cycles in bank conflicts)
    static constexpr bool BLK = W % 4 == 0 && W % 16 != 0 && TH % 8 == 0 && !(W == 24 && TH == 16 && NB == 1);
    static constexpr int RS = BLK ? W + 2 : W + 1, HR = TH + 2;  // halo row pitch (slots), rows
    // PM (pixel-major halo): a halo pixel's four 16-B planes are slots 5p .. 5p+3 (5p+4 is a
    // never-read pad), so a DMA instruction reads ~13 pixels x 64 contiguous bytes instead
    // of 64 pixels x 16 B (a quarter of the cache lines); the 80-B pixel pitch keeps 16
    // consecutive pixels' fragment reads on distinct banks.  Plane-major otherwise.
    static constexpr bool PM = PM_;
    static constexpr int HS = 1 + NB * HR * RS;                  // halo pixels (incl. the leading zero)
    static constexpr int HT = PM ? 5 * HS : 4 * HS;              // halo slots per chunk
    static constexpr int QSTRIDE = PM ? 1 : HS;                  // slots between planes of a pixel
    static constexpr int PSTRIDE = PM ? 5 : 1;                   // slots between pixels
    static constexpr int WT = 9 * 4 * BM;                        // weight slots per chunk
    static constexpr int ITEM_SLOTS = HT + (WRES ? 0 : WT);
    static constexpr int PPW = (ITEM_SLOTS + 64 * NW - 1) / (64 * NW);  // 1-KiB DMA pieces per wave per item
    static constexpr int BUF = PPW * NW * 1024;                  // bytes per ring slot
    static constexpr int WPPW = WRES ? (NCH * WT + 64 * NW - 1) / (64 * NW) : 0;  // resident weight pieces
    static constexpr int WOFF = 2 * BUF;                         // resident weight image
    static constexpr int LDS = 2 * BUF + WPPW * NW * 1024;
    static constexpr int STORES = 2 * NT;                        // epilogue stores per wave per tile
    static_assert(P == PG * NT * 32, "tile = pixel groups x 3 fragments x 32 pixels");
    static_assert(H % TH == 0 && CIN % 32 == 0, "tiling");
    static_assert((2 * QSTRIDE + (2 * RS + 2) * PSTRIDE) * 16 < 65536 && (36 * BM) * 16 < 65536,
                  "ds_read offset range");
    static_assert(STORES + 2 * NT < 64 && PPW < 64, "vmcnt range");
};

template <bool BLK, int W, int TH, int NB>
__device__ __forceinline__ int tile_pixel(int f, int r32) {
    if constexpr (BLK)
        return frag_pixel_blk<W, TH, NB>(f, r32);
    else
        return frag_pixel<W, TH, NB>(f, r32);
}

struct TParams {
    const uint16_t* x;
    const uint16_t* w;
    const float* bias;
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* zero;
    uint16_t* sink;
    int N, Cout, n_tiles, ncb;  // ncb = Cout / BM column blocks (1 when weights are resident)
};

template <int CIN, int H, int W, int TH, int NB, bool WRES, bool RES, int BM, bool PM>
__global__ __launch_bounds__(512, 1) void tconv_kernel(TParams p) {
    using G = TCfg<CIN, H, W, TH, NB, WRES, BM, PM>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int mg = wave % G::MG, pg = wave / G::MG;
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = H / TH;

    // weight slot (within one chunk's [tap][q][cout] image) -> element offset in w[cout][3][3][Cin]
    auto wsrc_off = [&](int ws) {
        const int tq = ws / G::BM, co = ws - (ws / G::BM) * G::BM;
        const int cs = (co & ~31) | row_cout(co & 31);
        return (cs * 9 + (tq >> 2)) * CIN + (tq & 3) * 8;
    };

    // ---- per-lane DMA geometry of this wave's item pieces (fixed for the launch)
    // pk: kind << 28 | nb << 8 | hy (kind 0 zero, 1 halo, 2 weight); po: element offset
    int pk[G::PPW], po[G::PPW];
#pragma unroll
    for (int j = 0; j < G::PPW; j++) {
        const int s = (j * G::NW + wave) * 64 + lane;  // slot within the ring slot
        int kind = 0, off = 0, nb = 0, hy = 0;
        if (s < G::HT) {
            const int q = PM ? s % 5 : s / G::HS, hs = PM ? s / 5 : s - (s / G::HS) * G::HS;
            if (hs > 0 && q < 4) {
                const int t = hs - 1;
                nb = t / (G::HR * G::RS);
                const int rr = t - nb * (G::HR * G::RS);
                hy = rr / G::RS;
                const int hx = rr - hy * G::RS;
                if (hx < W) {
                    kind = 1;
                    off = ((nb * H + hy - 1) * W + hx) * CIN + q * 8;  // from the tile's (crop, row 0, col 0)
                }
            }
        } else if (!WRES && s < G::HT + G::WT) {
            kind = 2;
            off = wsrc_off(s - G::HT);
        }
        pk[j] = (kind << 28) | (nb << 8) | hy;
        po[j] = off;
    }
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    auto tile_of = [&](int tile, int& n0, int& ho0, int& cb) {
        cb = tile % p.ncb;
        const int sp = tile / p.ncb;
        n0 = (sp / tiles_h) * NB;
        ho0 = (sp - (sp / tiles_h) * tiles_h) * TH;
    };
    auto issue = [&](int item, int buf) {
        const int tile = blockIdx.x + (item / G::NCH) * gridDim.x, chunk = item % G::NCH;
        int n0, ho0, cb;
        tile_of(tile, n0, ho0, cb);
        const uint16_t* xb = p.x + ((long)(n0 * H + ho0) * W) * CIN + chunk * 32;
        const uint16_t* wb = p.w + (long)cb * G::BM * 9 * CIN + chunk * 32;
        uint8_t* dst = lds + buf * G::BUF;
#pragma unroll
        for (int j = 0; j < G::PPW; j++) {
            const int g = pk[j], kind = g >> 28, nb = (g >> 8) & 255, hy = g & 255;
            const bool in = kind == 1 && (unsigned)(ho0 + hy - 1) < (unsigned)H && n0 + nb < p.N;
            const uint16_t* src = (!WRES && kind == 2) ? wb + po[j] : in ? xb + po[j] : zl;
            glds16(src, dst + (j * G::NW + wave) * 1024);
        }
    };

    // ---- fragment base addresses (bytes) and output geometry
    int bv[G::NT], eoff[G::NT], enb[G::NT];
#pragma unroll
    for (int t = 0; t < G::NT; t++) {
        const int pp = tile_pixel<G::BLK, W, TH, NB>(pg * G::NT + t, r32);
        const int nb = pp / (TH * W), rem = pp - nb * (TH * W);
        const int ty = rem / W, x = rem - (rem / W) * W;
        bv[t] = (h * G::QSTRIDE + (nb * G::HR * G::RS + ty * G::RS + x) * G::PSTRIDE) * 16;
        eoff[t] = (nb * H + ty) * W + x;  // output pixel from the tile's (n0, ho0, 0)
        enb[t] = nb;
    }
    // A fragment row r32 of cout group mg, k half h
    const int av = WRES ? G::WOFF + (h * G::BM + mg * 32 + r32) * 16 : (G::HT + h * G::BM + mg * 32 + r32) * 16;

    const int n_items = ((p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) * G::NCH;
    // The lane's 16 folded-BN biases, loaded ONCE: a workgroup's tiles all have the same
    // column block (tile = blockIdx.x + k * gridDim.x and gridDim.x % ncb == 0, checked by
    // the launcher).  Initialising the accumulators from a per-tile global load made the
    // compiler wait for ALL outstanding VMEM (vmcnt(0): the next item's DMA, issued after
    // it) before the tile's first MFMA; from LDS, it waited for the previous tile's stores
    // (a conservative LDS-DMA alias wait before the read).
    f32x16 bias_init;
    {
        const float* bp = p.bias + (blockIdx.x % p.ncb) * G::BM + mg * 32 + 16 * h;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float4 b4 = *reinterpret_cast<const float4*>(bp + 4 * j);
            bias_init[4 * j] = b4.x;
            bias_init[4 * j + 1] = b4.y;
            bias_init[4 * j + 2] = b4.z;
            bias_init[4 * j + 3] = b4.w;
        }
    }
    if (WRES) {  // all weight chunks, once (column block 0: host guarantees ncb == 1)
#pragma unroll
        for (int j = 0; j < G::WPPW; j++) {
            const int s = (j * G::NW + wave) * 64 + lane;
            const int chunk = s / G::WT;
            const uint16_t* src = s < G::NCH * G::WT ? p.w + chunk * 32 + wsrc_off(s - chunk * G::WT) : zl;
            glds16(src, lds + G::WOFF + (j * G::NW + wave) * 1024);
        }
    }
    issue(0, 0);
    f32x16 acc[G::NT];
    for (int k = 0; k < n_items; k++) {
        const int buf = k & 1, chunk = k % G::NCH;
        const bool first = chunk == 0, last = chunk == G::NCH - 1;
        // item k's DMA has landed (younger: only the previous tile's stores); the barrier
        // publishes all waves' pieces and retires every read of the other ring slot
        if (k == 0 || !first)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::STORES) : "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int tile = blockIdx.x + (k / G::NCH) * gridDim.x;
        int n0, ho0, cb;
        tile_of(tile, n0, ho0, cb);
        const int cob = cb * G::BM + mg * 32 + 16 * h;  // this lane's 16 couts
        if (first) {
#pragma unroll
            for (int t = 0; t < G::NT; t++) acc[t] = bias_init;
        }
        // residual of this tile (last item), issued before the next DMA so that the
        // epilogue's wait never waits for it
        uint4 rv[G::NT][2];
        const long pix0 = (long)(n0 * H + ho0) * W;
        if (RES && last) {
#pragma unroll
            for (int t = 0; t < G::NT; t++) {
                const bool ok = n0 + enb[t] < p.N;
                const uint16_t* rs = ok ? p.res + (pix0 + eoff[t]) * p.Cout + cob : p.zero + lane * 16;
                rv[t][0] = *reinterpret_cast<const uint4*>(rs);
                rv[t][1] = *reinterpret_cast<const uint4*>(rs + 8);
            }
        }
        asm volatile("" ::: "memory");
        const bool more = k + 1 < n_items;
        // unconditional (the last item re-fetches itself into the idle slot): a branch around
        // the DMA made the compiler fall back to vmcnt(0) — waiting for this DMA — before the
        // residual's first use in the epilogue
        issue(more ? k + 1 : k, buf ^ 1);
        asm volatile("" ::: "memory");

        // ---- 9 taps x 2 k-steps x NT MFMAs; fragments of step s+1 read before step s's MFMAs
        const int boff = buf * G::BUF;
        int bva[G::NT];
#pragma unroll
        for (int t = 0; t < G::NT; t++) bva[t] = bv[t] + boff;
        const int ava = WRES ? av + chunk * G::WT * 16 : av + boff;
        // fragments of step s+LD are read before step s's MFMAs (LD = LDS read look-ahead; 2
        // measured level with 1: the loop is not LDS-latency bound)
        constexpr int LD = 1, NBF = LD + 1;
        bf16x8 fa[NBF], fb[NBF][G::NT];
        auto load = [&](int step, bf16x8& a, bf16x8 (&b)[G::NT]) {
            const int tap = step >> 1, ks = step & 1;
            const int dy = tap / 3, dx = tap % 3;
            a = *reinterpret_cast<const bf16x8*>(lds + ava + (tap * 4 + ks * 2) * G::BM * 16);
#pragma unroll
            for (int t = 0; t < G::NT; t++)
                b[t] = *reinterpret_cast<const bf16x8*>(lds + bva[t] +
                                                        (ks * 2 * G::QSTRIDE + (dy * G::RS + dx) * G::PSTRIDE) * 16);
        };
#pragma unroll
        for (int s0 = 0; s0 < LD; s0++) load(s0, fa[s0], fb[s0]);
#pragma unroll
        for (int step = 0; step < 18; step++) {
            const int cur = step % NBF;
            if (step + LD < 18) load(step + LD, fa[(step + LD) % NBF], fb[(step + LD) % NBF]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < G::NT; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        if (last) {
            if (RES) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::PPW) : "memory");
#pragma unroll
            for (int t = 0; t < G::NT; t++) {
                const bool ok = n0 + enb[t] < p.N;
                uint16_t* yrow = ok ? p.y + (pix0 + eoff[t]) * p.Cout + cob : p.sink + lane * 16;
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    float v0 = acc[t][2 * e], v1 = acc[t][2 * e + 1];
                    if (RES) {
                        const uint4 rr = rv[t][e >> 2];
                        const uint32_t u = (e & 3) == 0 ? rr.x : (e & 3) == 1 ? rr.y : (e & 3) == 2 ? rr.z : rr.w;
                        v0 += lo_bf16(u);
                        v1 += hi_bf16(u);
                    }
                    o[e] = pack_bf16x2(relu1(v0), relu1(v1));
                }
                *reinterpret_cast<uint4*>(yrow) = uint4{o[0], o[1], o[2], o[3]};
                *reinterpret_cast<uint4*>(yrow + 8) = uint4{o[4], o[5], o[6], o[7]};
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int g_t_cus = 0;
uint16_t* g_t_sink = nullptr;

template <int CIN, int H, int W, int TH, int NB, bool WRES, bool RES, int BM, bool PM>
void launch_t_kernel(const TParams& p, hipStream_t s) {
    using G = TCfg<CIN, H, W, TH, NB, WRES, BM, PM>;
    static_assert(G::LDS <= 160 * 1024, "LDS budget");
    auto kern = tconv_kernel<CIN, H, W, TH, NB, WRES, RES, BM, PM>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    const int grid = std::min(p.n_tiles, g_t_cus);
    MVP_REQUIRE(grid % p.ncb == 0, "tconv: grid %d not a multiple of the %d column blocks", grid, p.ncb);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT_THREADS), G::LDS, s, p);
}

template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM = 64>
void launch_t(const ConvLaunch& c, hipStream_t s) {
    if (g_t_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_t_cus, hipDeviceAttributeMultiprocessorCount, dev));
        MVP_HIP(hipMalloc(&g_t_sink, 64 * 32));
    }
    MVP_REQUIRE(!WRES || c.Cout == BM, "tconv: resident weights need Cout == BM");
    MVP_REQUIRE(c.Cout % BM == 0, "tconv: Cout %d not a multiple of %d", c.Cout, BM);
    const long tiles = (long)((c.N + NB - 1) / NB) * (H / TH) * (c.Cout / BM);
    MVP_REQUIRE(tiles < (1L << 30), "tconv: too many tiles");
    TParams p{c.x, c.w, c.bias, c.res, c.y, conv_zero_region(), g_t_sink, c.N, c.Cout, (int)tiles, c.Cout / BM};
    // pixel-major halo wherever its 25 % larger ring slot still fits the LDS (+2.4-2.9 %
    // frames/s on the 64- and 256-ch planes, round 2), plane-major otherwise
    constexpr bool PM = TCfg<CIN, H, W, TH, NB, WRES, BM, true>::LDS <= 160 * 1024;
    if (c.res)
        launch_t_kernel<CIN, H, W, TH, NB, WRES, true, BM, PM>(p, s);
    else
        launch_t_kernel<CIN, H, W, TH, NB, WRES, false, BM, PM>(p, s);
}

}  // namespace

bool launch_tconv(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 3 || c.stride != 1 || c.out_f32_nchw || !c.relu || c.Cout % 32 != 0) return false;
    const char* e = getenv("MVPOSE_NO_TCONV");  // diagnostics/tests: fall back to the other kernels
    if (e && e[0] == '1') return false;
    // transition1.0: 256 -> 32 @ 64x48, 32-cout tiles of 768 pixels (8 pixel groups), streamed weights
    if (c.Cin == 256 && c.Cout == 32 && c.H == 64 && c.W == 48) {
        launch_t<256, 64, 48, 16, 1, false, 32>(c, s);
        return true;
    }
    if (c.Cout % 64 != 0) return false;
    if (c.Cin == 64 && c.Cout == 64 && c.H == 32 && c.W == 24) {
        launch_t<64, 32, 24, 16, 1, true>(c, s);
        return true;
    }
    if (c.Cin == 64 && c.Cout == 64 && c.H == 64 && c.W == 48) {
        launch_t<64, 64, 48, 8, 1, true>(c, s);
        return true;
    }
    if (launch_tconv16(c, s)) return true;  // 128 ch @ 16x12, 256 ch @ 8x6: 128-cout tiles
    // 128 ch @ 16x12 without a weight image (streamed weights, two crops per tile; the
    // weight-stationary wsconv.hip it replaced in round 2 measured 86.2 us/conv against this
    // kernel's 87.9 on the plane-major halo, 10,207 -> 10,479 frames/s with the pixel-major one)
    if (c.Cin == 128 && c.H == 16 && c.W == 12) {
        launch_t<128, 16, 12, 16, 2, false>(c, s);
        return true;
    }
    if (c.Cin == 256 && c.H == 8 && c.W == 6) {
        launch_t<256, 8, 6, 8, 8, false>(c, s);
        return true;
    }
    return false;
}

}  // namespace mvp
