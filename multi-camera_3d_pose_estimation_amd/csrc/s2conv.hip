// 3x3 / stride-2 implicit-GEMM convolution on v_mfma_f32_32x32x16_bf16 (gfx950).
//
// HRNet-W32's stride-2 convs (stem conv2, the transitions to a new branch, the
// downsampling fuse-layer chains) ran on the generic conv_mfma_kernel at 4-12 % of
// the MFMA peak (5.4 ms of a 31 ms forward at 1024 crops; the 8x6-output ones on a
// masked 4x16 tiling that wasted 60 % of each tile).
// This kernel is tconv.hip's design transposed to stride 2:
//
//  * Polyphase halo.  The input rows/cols a tile needs are split into their four
//    (row parity, col parity) phases, each stored as a plane of (TH+1) x (WO+1)
//    16-B slots (WO = output width).  Output pixel (y, x), tap (dy, dx) reads phase
//    (dy & 1, dx & 1) at (y + dy/2, x + dx/2): one base VGPR per fragment plus a
//    compile-time immediate per tap, and the 16 lanes of a ds_read_b128 group read 16
//    consecutive slots (no stride-2 bank conflicts).  Phase (0, 0) column 0 and row 0
//    of the first tile are the zero padding.
//  * 16-channel items.  A stride-2 tile needs 4x the input pixels of a stride-1 tile
//    of the same output, so one work item is (tile, 16 input channels): two 8-channel
//    planes of halo plus that slice of the weights ([tap][plane][cout]), double
//    buffered by LDS-DMA (global_load_lds) while the previous item computes (9 MFMAs
//    per fragment per item, one per tap).  Cin = 32 convs keep all their weights
//    resident in LDS instead.
//  * Accumulators start at the folded-BN bias; ReLU (optional: the last conv of a
//    fuse-layer chain has none) and bf16 packing fused; permuted couts as in tconv
//    (row_cout), so each lane stores 2 x 16 B per fragment.
// 8 waves (2 per SIMD) per workgroup, one workgroup per CU, persistent over tiles.
// K order is (16-channel slice, tap, channel): results agree with the other conv
// kernels to f32 summation-order rounding.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;  // 16-B slots of the shared zero region

template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM, bool PM_ = false>
struct SCfg {
    static constexpr int NW = 8, NT_THREADS = NW * 64;
    static constexpr int MG = BM / 32, PG = NW / MG;  // cout groups x pixel groups
    static constexpr int NT = 3;                      // 32-pixel fragments per wave
    static constexpr int HO = H / 2, WO = W / 2;
    static constexpr int P = NB * TH * WO;            // output pixels per tile
    static constexpr int NCH = CIN / 16;              // items per tile
    static constexpr int RS = WO + 1, HR = TH + 1;    // phase-plane row pitch (slots), rows
    static constexpr int PH = HR * RS;                // slots per phase plane
    static constexpr int HS = NB * 4 * PH;            // halo pixels per item
    static constexpr int HT = 2 * HS;                 // halo slots per item
    // PM (pixel-major halo): a pixel's two 16-B planes are adjacent slots (32 B contiguous per
    // pixel in a DMA instruction, half the cache lines of plane-major) at the price of 2-way
    // bank conflicts on the fragment reads (16 pixels x 32 B pitch); plane-major otherwise.
    static constexpr bool PM = PM_;
    static constexpr int QS = PM ? 1 : HS, PS = PM ? 2 : 1;  // slots between planes / pixels
    static constexpr int WT = 9 * 2 * BM;             // weight slots per item
    static constexpr int ITEM_SLOTS = HT + (WRES ? 0 : WT);
    static constexpr int PPW = (ITEM_SLOTS + 64 * NW - 1) / (64 * NW);  // 1-KiB DMA pieces per wave per item
    static constexpr int BUF = PPW * NW * 1024;
    static constexpr int WPPW = WRES ? (NCH * WT + 64 * NW - 1) / (64 * NW) : 0;
    static constexpr int WOFF = 2 * BUF;
    static constexpr int LDS = 2 * BUF + WPPW * NW * 1024;
    static constexpr int STORES = 2 * NT;
    static_assert(P == PG * NT * 32, "tile = pixel groups x 3 fragments x 32 pixels");
    static_assert(H % 2 == 0 && W % 2 == 0 && HO % TH == 0 && CIN % 16 == 0, "tiling");
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert((QS + (3 * PH + RS + 1) * PS) * 16 < 65536 && (16 * BM + 2 * BM) * 16 < 65536,
                  "ds_read offset range");
    static_assert(STORES < 64 && 2 * PPW < 64, "vmcnt range");
    static_assert(2 * TH + 1 < 256, "row index packing");
};

struct SParams {
    const uint16_t* x;
    const uint16_t* w;
    const float* bias;
    uint16_t* y;
    const uint16_t* zero;
    uint16_t* sink;
    int N, Cout, n_tiles, ncb, relu;
    // sibling outputs (graph sib-fusion): couts [Cout, Cout + c1) go to y1 ([..][c1]) and
    // [Cout + c1, Cout + c1 + c2) to y2, each with its own ReLU flag; couts beyond are padding
    uint16_t* y1;
    uint16_t* y2;
    int c1, c2, relu1, relu2;
    int img;  // w is the slot-order weight image (tconv16_pack_weights, BM = 128): 1 KB contiguous per DMA piece
};

template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM, bool PM>
__global__ __launch_bounds__(512, 1) void s2conv_kernel(SParams p) {
    using G = SCfg<CIN, H, W, TH, NB, WRES, BM, PM>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int mg = wave % G::MG, pg = wave / G::MG;
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = G::HO / TH;

    // weight slot (within one item's [tap][plane][cout] image) -> element offset in
    // w[cout][3][3][Cin] from the item's first channel
    auto wsrc_off = [&](int ws) {
        const int tq = ws / BM, co = ws - (ws / BM) * BM;
        const int cs = (co & ~31) | row_cout(co & 31);
        return (cs * 9 + (tq >> 1)) * CIN + (tq & 1) * 8;
    };

    // ---- per-lane DMA geometry (fixed for the launch)
    // pk: kind << 28 | nb << 8 | hy (kind 0 zero, 1 halo, 2 weight; hy = input row - 2*ho0 + 1).
    // Streamed-weight planes (!WRES): waves 0-3 issue the item pieces of virtual waves vw = wave
    // and wave + 4 (their SIMD partner), waves 4-7 none: after the item barrier one wave per
    // SIMD starts its MFMAs at once while the other issues the DMA (tconv16.hip; 4-6 % per
    // launch, profiles/r04_dma_split_ab.txt).  The resident-weight planes (halo-only items)
    // measured level to 2 % slower that way, so every wave issues its own pieces there.
    constexpr bool SPLIT = !WRES;
    constexpr int NVW = SPLIT ? 2 : 1;
    const bool dma_wave = !SPLIT || wave < 4;
    auto vwave = [&](int v) { return SPLIT ? (wave & 3) + 4 * v : wave; };
    int pk[NVW][G::PPW], po[NVW][G::PPW];
#pragma unroll
    for (int v = 0; v < NVW; v++)
#pragma unroll
    for (int j = 0; j < G::PPW; j++) {
        const int s = (j * G::NW + vwave(v)) * 64 + lane;
        int kind = 0, off = 0, nb = 0, hy = 0;
        if (s < G::HT) {
            const int qh = PM ? s & 1 : s / G::HS, hs = PM ? s >> 1 : s - (s / G::HS) * G::HS;
            nb = hs / (4 * G::PH);
            const int rem = hs - nb * (4 * G::PH);
            const int ph = rem / G::PH, rr = rem - (rem / G::PH) * G::PH;
            const int a = rr / G::RS, b = rr - (rr / G::RS) * G::RS;
            hy = 2 * a + (ph >> 1);
            const int col = 2 * b + (ph & 1) - 1;
            if (col >= 0 && col < W) {
                kind = 1;
                off = ((nb * H + hy - 1) * W + col) * CIN + qh * 8;  // from the tile's (crop, row 2*ho0, col 0)
            }
        } else if (!WRES && s < G::HT + G::WT) {
            kind = 2;
            off = p.img ? (s - G::HT) * 8 : wsrc_off(s - G::HT);
        }
        pk[v][j] = (kind << 28) | (nb << 8) | hy;
        po[v][j] = off;
    }
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    auto tile_of = [&](int tile, int& n0, int& ho0, int& cb) {
        cb = tile % p.ncb;
        const int sp = tile / p.ncb;
        n0 = (sp / tiles_h) * NB;
        ho0 = (sp - (sp / tiles_h) * tiles_h) * TH;
    };
    auto issue = [&](int item, int buf) {
        const int tile = blockIdx.x + (item / G::NCH) * gridDim.x, slice = item % G::NCH;
        int n0, ho0, cb;
        tile_of(tile, n0, ho0, cb);
        const uint16_t* xb = p.x + ((long)(n0 * H + 2 * ho0) * W) * CIN + slice * 16;
        const uint16_t* wb =
            p.img ? p.w + (long)(cb * G::NCH + slice) * G::WT * 8 : p.w + (long)cb * BM * 9 * CIN + slice * 16;
        uint8_t* dst = lds + buf * G::BUF;
        if (!dma_wave) return;
#pragma unroll
        for (int v = 0; v < NVW; v++)
#pragma unroll
        for (int j = 0; j < G::PPW; j++) {
            const int vw = vwave(v);
            const int g = pk[v][j], kind = g >> 28, nb = (g >> 8) & 255, hy = g & 255;
            const bool in = kind == 1 && (unsigned)(2 * ho0 + hy - 1) < (unsigned)H && n0 + nb < p.N;
            const uint16_t* src = (!WRES && kind == 2) ? wb + po[v][j] : in ? xb + po[v][j] : zl;
            // pieces wholly past the item's slots are not issued (the 128->256 plane: 4 of 72)
            if (j < G::PPW - 1 || (j * G::NW + vw) * 64 < G::ITEM_SLOTS)
                glds16(src, dst + (j * G::NW + vw) * 1024);
        }
    };

    // ---- fragment base addresses (bytes) and output geometry
    int bv[G::NT], eoff[G::NT], enb[G::NT];
#pragma unroll
    for (int t = 0; t < G::NT; t++) {
        const int pp = frag_pixel<G::WO, TH, NB>(pg * G::NT + t, r32);
        const int nb = pp / (TH * G::WO), rem = pp - nb * (TH * G::WO);
        const int ty = rem / G::WO, x = rem - (rem / G::WO) * G::WO;
        bv[t] = (h * G::QS + (nb * 4 * G::PH + ty * G::RS + x) * G::PS) * 16;
        eoff[t] = (nb * G::HO + ty) * G::WO + x;
        enb[t] = nb;
    }
    const int av = WRES ? G::WOFF + (h * BM + mg * 32 + r32) * 16 : (G::HT + h * BM + mg * 32 + r32) * 16;

    const int n_items = ((p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) * G::NCH;
    if (WRES) {  // all weight slices, once (host guarantees ncb == 1)
#pragma unroll
        for (int j = 0; j < G::WPPW; j++) {
            const int s = (j * G::NW + wave) * 64 + lane;
            const int slice = s / G::WT;
            const uint16_t* src = s < G::NCH * G::WT ? p.w + slice * 16 + wsrc_off(s - slice * G::WT) : zl;
            glds16(src, lds + G::WOFF + (j * G::NW + wave) * 1024);
        }
    }
    issue(0, 0);
    f32x16 acc[G::NT];
    for (int k = 0; k < n_items; k++) {
        const int buf = k & 1, slice = k % G::NCH;
        const bool first = slice == 0, last = slice == G::NCH - 1;
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
        const int cob = cb * BM + mg * 32 + 16 * h;  // this lane's 16 couts
        if (first) {
            f32x16 b;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float4 b4 = *reinterpret_cast<const float4*>(p.bias + cob + 4 * j);
                b[4 * j] = b4.x;
                b[4 * j + 1] = b4.y;
                b[4 * j + 2] = b4.z;
                b[4 * j + 3] = b4.w;
            }
#pragma unroll
            for (int t = 0; t < G::NT; t++) acc[t] = b;
        }
        const bool more = k + 1 < n_items;
        if (more) issue(k + 1, buf ^ 1);
        asm volatile("" ::: "memory");

        // ---- 9 taps x NT MFMAs; fragments of tap s+1 read before tap s's MFMAs
        const int boff = buf * G::BUF;
        int bva[G::NT];
#pragma unroll
        for (int t = 0; t < G::NT; t++) bva[t] = bv[t] + boff;
        const int ava = WRES ? av + slice * G::WT * 16 : av + boff;
        bf16x8 fa[2], fb[2][G::NT];
        auto load = [&](int tap, bf16x8& a, bf16x8 (&b)[G::NT]) {
            const int dy = tap / 3, dx = tap % 3;
            const int toff = ((dy & 1) * 2 + (dx & 1)) * G::PH + (dy >> 1) * G::RS + (dx >> 1);
            a = *reinterpret_cast<const bf16x8*>(lds + ava + tap * 2 * BM * 16);
#pragma unroll
            for (int t = 0; t < G::NT; t++) b[t] = *reinterpret_cast<const bf16x8*>(lds + bva[t] + toff * G::PS * 16);
        };
        load(0, fa[0], fb[0]);
#pragma unroll
        for (int tap = 0; tap < 9; tap++) {
            const int cur = tap & 1;
            if (tap + 1 < 9) load(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < G::NT; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        if (last) {
            const long pix0 = (long)(n0 * G::HO + ho0) * G::WO;
            // which output this lane's 16 couts belong to (boundaries are multiples of 32)
            uint16_t* yb = p.y;
            int cs = p.Cout, cl = cob, rl = p.relu;
            bool cok = true;
            if (cob >= p.Cout) {
                const bool s1 = cob < p.Cout + p.c1;
                yb = s1 ? p.y1 : p.y2;
                cs = s1 ? p.c1 : p.c2;
                cl = s1 ? cob - p.Cout : cob - p.Cout - p.c1;
                rl = s1 ? p.relu1 : p.relu2;
                cok = cob < p.Cout + p.c1 + p.c2;
            }
#pragma unroll
            for (int t = 0; t < G::NT; t++) {
                const bool ok = n0 + enb[t] < p.N && cok;
                uint16_t* yrow = ok ? yb + (pix0 + eoff[t]) * cs + cl : p.sink + lane * 16;
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    float v0 = acc[t][2 * e], v1 = acc[t][2 * e + 1];
                    if (rl) {
                        v0 = relu1(v0);
                        v1 = relu1(v1);
                    }
                    o[e] = pack_bf16x2(v0, v1);
                }
                *reinterpret_cast<uint4*>(yrow) = uint4{o[0], o[1], o[2], o[3]};
                *reinterpret_cast<uint4*>(yrow + 8) = uint4{o[4], o[5], o[6], o[7]};
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int g_s_cus = 0;
uint16_t* g_s_sink = nullptr;

template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM, bool PM>
void launch_sp_pm(SParams p, hipStream_t s) {
    using G = SCfg<CIN, H, W, TH, NB, WRES, BM, PM>;
    auto kern = s2conv_kernel<CIN, H, W, TH, NB, WRES, BM, PM>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    const int grid = std::min(p.n_tiles, g_s_cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT_THREADS), G::LDS, s, p);
}

// the pixel-major halo (+0.7 % frames/s over plane-major, round 2)
template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM>
void launch_sp(SParams p, hipStream_t s) {
    launch_sp_pm<CIN, H, W, TH, NB, WRES, BM, true>(p, s);
}

template <int CIN, int H, int W, int TH, int NB, bool WRES, int BM>
void launch_s(const ConvLaunch& c, hipStream_t s) {
    using G = SCfg<CIN, H, W, TH, NB, WRES, BM>;
    if (g_s_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_s_cus, hipDeviceAttributeMultiprocessorCount, dev));
        MVP_HIP(hipMalloc(&g_s_sink, 64 * 32));
    }
    MVP_REQUIRE(!WRES || c.Cout == BM, "s2conv: resident weights need Cout == BM");
    MVP_REQUIRE(c.Cout % BM == 0, "s2conv: Cout %d not a multiple of %d", c.Cout, BM);
    MVP_REQUIRE(c.Cin == CIN && c.H == H && c.W == W, "s2conv: plane mismatch");
    const long tiles = (long)((c.N + NB - 1) / NB) * (G::HO / TH) * (c.Cout / BM);
    MVP_REQUIRE(tiles < (1L << 30), "s2conv: too many tiles");
    // streamed weights from the graph's weight image when it made one (BM = 128 layout)
    const bool img = !WRES && BM == 128 && c.w_img != nullptr;
    SParams p{c.x, img ? c.w_img : c.w, c.bias, c.y, conv_zero_region(), g_s_sink, c.N, c.Cout, (int)tiles,
              c.Cout / BM, c.relu, nullptr, nullptr, 0, 0, 0, 0, img ? 1 : 0};
    launch_sp<CIN, H, W, TH, NB, WRES, BM>(p, s);
}

void init_s() {
    if (g_s_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_s_cus, hipDeviceAttributeMultiprocessorCount, dev));
        MVP_HIP(hipMalloc(&g_s_sink, 64 * 32));
    }
}

}  // namespace

bool s2conv_multi_supported(int H, int W, int Cin, int total_cout) {
    const char* e = getenv("MVPOSE_NO_SIBFUSE");  // diagnostics/tests: one launch per sibling
    if (e && e[0] == '1') return false;
    return H == 64 && W == 48 && Cin == 32 && total_cout <= 128;
}

// The sibling 3x3/s2 convs reading the 64x48x32 branch-0 tensor in a fuse layer (-> 64 ch
// for branch 1, -> 32 ch (ReLU) starting the chains to branches 2 and 3): one launch, one
// pass over the input, 128-cout tiles (weights concatenated along cout, zero-padded).
void launch_s2conv_multi(const S2Multi& m, hipStream_t s) {
    MVP_REQUIRE(m.n_out >= 1 && m.n_out <= 3, "s2conv_multi: %d outputs", m.n_out);
    int tot = 0;
    for (int i = 0; i < m.n_out; i++) {
        MVP_REQUIRE(m.cout[i] % 32 == 0 && m.cout[i] > 0, "s2conv_multi: cout %d", m.cout[i]);
        tot += m.cout[i];
    }
    MVP_REQUIRE(s2conv_multi_supported(m.H, m.W, m.Cin, tot), "s2conv_multi: unsupported plane");
    init_s();
    using G = SCfg<32, 64, 48, 8, 1, true, 128>;
    const long tiles = (long)m.N * (G::HO / 8);
    SParams p{m.x, m.w, m.bias, m.y[0], conv_zero_region(), g_s_sink, m.N, m.cout[0], (int)tiles, 1, m.relu[0],
              m.n_out > 1 ? m.y[1] : nullptr, m.n_out > 2 ? m.y[2] : nullptr, m.n_out > 1 ? m.cout[1] : 0,
              m.n_out > 2 ? m.cout[2] : 0, m.n_out > 1 ? m.relu[1] : 0, m.n_out > 2 ? m.relu[2] : 0, 0};
    if (tiles == 0) return;
    launch_sp<32, 64, 48, 8, 1, true, 128>(p, s);
    MVP_HIP(hipGetLastError());
}

bool launch_s2conv(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 3 || c.stride != 2 || c.out_f32_nchw || c.res || c.x2) return false;
    const char* e = getenv("MVPOSE_NO_S2CONV");  // diagnostics/tests: fall back to conv_mfma_kernel
    if (e && e[0] == '1') return false;
    const int ci = c.Cin, co = c.Cout, h = c.H, w = c.W;
    // Planes where the 16-channel items lose to conv_mfma_kernel stay there (tools/s2_bench.py,
    // 1024 crops): stem conv2 64@128x96 (1415 vs 796 us), transition1.1 256@64x48 (1162 vs
    // 1057 us) and 64->64 @32x24 (80 vs 51 us).  Their items carry 16 of a pixel's 64..256
    // channels, so each 128-B line is fetched once per item: L2 cannot hold a tile's lines
    // across its 4..16 items and the gather over-fetches 4x.
    if (h == 64 && w == 48 && co == 64 && ci == 32)  // fuse 1<-0
        return launch_s<32, 64, 48, 16, 1, true, 64>(c, s), true;
    if (h == 32 && w == 24 && co == 128) {  // transition2, fuse 2<-{0,1}
        if (ci == 32) return launch_s<32, 32, 24, 16, 1, true, 128>(c, s), true;
        if (ci == 64) return launch_s<64, 32, 24, 16, 1, false, 128>(c, s), true;
    }
    if (h == 16 && w == 12 && co % 128 == 0) {  // -> 256 @ 8x6: transition3, fuse 3<-{0,1,2}
        if (ci == 32) return launch_s<32, 16, 12, 8, 4, false, 128>(c, s), true;
        if (ci == 64) return launch_s<64, 16, 12, 8, 4, false, 128>(c, s), true;
        if (ci == 128) return launch_s<128, 16, 12, 8, 4, false, 128>(c, s), true;
    }
    return false;
}

}  // namespace mvp
