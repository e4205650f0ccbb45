// 3x3/s1 implicit-GEMM convolution for the low-resolution HRNet-W32 branch planes
// (128 ch @ 16x12 and 256 ch @ 8x6) on v_mfma_f32_32x32x16_bf16 (gfx950).
//
// tconv.hip's items are (384-pixel x 64-cout tile, 32 cin): for these planes the weights
// do not fit the LDS, so every item streams a 37 KB weight slice plus a 40 KB halo, and
// each wave reads 4 LDS fragments per 3 MFMAs.  Diagnostics on that kernel (MVPOSE_TCONV_DIAG,
// profiles/r03t128_diag.txt) showed the MFMA work and the LDS-read / DMA work adding up
// instead of overlapping (61.6 us per conv without DMA or stores; 40.3 us with a third of
// the MFMAs).  Here an item is (384 pixels x 128 couts, 16 cin):
//
//  * a wave owns 64 couts x 96 pixels (2 A x 3 B fragments): 5 ds_read_b128 per 6 MFMAs
//    (0.83 per MFMA instead of 1.33);
//  * 128 couts per tile: the 128-ch plane reads its halo once instead of per 64-cout
//    block; per item 53-62 KB of DMA (8 pieces per wave) for the same 54 MFMAs per wave
//    (10 pieces before);
//  * halo pixels at a 48-B pitch (two 16-B planes + a never-read pad slot; row pitch
//    W + 1, crop pitch (TH + 2)(W + 1)) and a lane -> pixel map (HMap) that gives the 16
//    lanes of each ds_read_b128 lane group 16 pixels of distinct slot residues mod 16:
//    conflict-free fragment reads for any tap (the 8x6 plane's raster map had 2-way
//    conflicts on every B read);
//  * the two 128-cout halves of a 256-ch tile run on the same XCD at the same time
//    (tile -> (spatial tile, cout block) is XCD-major), so the second halo read hits L2.
// Everything else follows tconv.hip: a two-slot LDS-DMA ring one item ahead, accumulators
// initialised to the folded-BN bias, fused residual + ReLU + bf16 epilogue with each lane
// owning 16 consecutive couts of its pixel, 8 waves, one persistent workgroup per CU.
// K order (16-cin chunk, tap, cin): f32 summation-order differences from tconv only.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots16 = 4096;

template <int CIN, int H, int W, int TH, int NB, int BM>
struct T16Cfg {
    static constexpr int NW = 8, NT_THREADS = NW * 64;
    static constexpr int MG = BM / 64, PG = NW / MG;  // 64-cout groups x pixel groups
    static constexpr int NT = 3;                      // 32-pixel B fragments per wave
    static constexpr int NA = 2;                      // 32-cout A fragments per wave
    static constexpr int P = NB * TH * W;             // output pixels per tile
    static constexpr int NCH = CIN / 16;              // items per tile
    static constexpr int RS = W + 1, HR = TH + 2, CS = HR * RS;
    static constexpr int HS = 1 + NB * CS;             // halo pixels (incl. the leading zero)
    static constexpr int HT = 3 * HS;                  // halo slots (48-B pixel pitch)
    static constexpr int WT = 9 * 2 * BM;              // weight slots [tap][q][cout]
    static constexpr int PPW = (HT + WT + 64 * NW - 1) / (64 * NW);
    static constexpr int BUF = PPW * NW * 1024;
    static constexpr int BIAS_OFF = 2 * BUF;                     // BM f32 folded-BN biases
    static constexpr int LDS = 2 * BUF + BM * 4;
    static constexpr int STORES = 2 * NA * NT;
    static_assert(P == PG * NT * 32 && NW % MG == 0, "tile = pixel groups x 3 fragments x 32 pixels");
    static_assert(H % TH == 0 && CIN % 16 == 0, "tiling");
    static_assert(((2 * RS + 2) * 3 + 1) * 16 < 65536 && (18 * BM) * 16 < 65536, "ds_read offset range");
    static_assert(STORES + 2 * NA * NT < 64 && 2 * PPW < 64, "vmcnt range");
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(NB <= 31 && HR <= 31 && (long)BM * 9 * CIN < (1 << 19) && (long)NB * H * W * CIN < (1 << 19),
                  "DMA geometry packing");
};

// Lane -> tile pixel map.  Fragment f's lane group g (= lane_grp) position pos (= lane_pos)
// takes the (2f + g)-th pixel (raster order) whose halo slot residue (3 * halo pixel mod 16;
// 3 is odd, so the pixel index mod 16) equals pos: each group's 16 pixels then sit on 16
// distinct residues, for every tap (a tap adds the same offset to all of them).  Needs every
// residue class to hold exactly P / 16 pixels (static_assert'ed).
template <int H, int W, int TH, int NB>
struct HMap {
    static constexpr int P = NB * TH * W, RS = W + 1, CS = (TH + 2) * RS;
    short pix[P];
    constexpr HMap() : pix() {
        int cnt[16] = {};
        for (int pp = 0; pp < P; pp++) {
            const int nb = pp / (TH * W), rem = pp % (TH * W), y = rem / W, x = rem % W;
            const int r = (nb * CS + y * RS + x) % 16;
            pix[cnt[r] * 16 + r] = (short)pp;
            cnt[r]++;
        }
    }
    constexpr bool balanced() const {
        int cnt[16] = {};
        for (int pp = 0; pp < P; pp++) {
            const int nb = pp / (TH * W), rem = pp % (TH * W), y = rem / W, x = rem % W;
            cnt[(nb * CS + y * RS + x) % 16]++;
        }
        for (int r = 0; r < 16; r++)
            if (cnt[r] != P / 16) return false;
        return true;
    }
};

template <int H, int W, int TH, int NB>
__device__ const HMap<H, W, TH, NB> kHMap{};

struct T16Params {
    const uint16_t* x;
    const uint16_t* w;  // weight image (tconv16_pack_weights)
    const float* bias;
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* zero;
    uint16_t* sink;
    int N, Cout, n_tiles, ncb;
};

template <int CIN, int H, int W, int TH, int NB, int BM, bool RES>
__global__ __launch_bounds__(512, 1) void tconv16_kernel(T16Params p) {
    using G = T16Cfg<CIN, H, W, TH, NB, BM>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int mg = wave % G::MG, pg = wave / G::MG;
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = H / TH;

    // ---- per-lane DMA geometry (fixed for the launch): kind << 29 | nb << 24 | hy << 19 | offset.
    // Waves 0-3 issue the pieces of "virtual waves" vw = wave and wave + 4 (their SIMD partner),
    // waves 4-7 issue none: after the item barrier one wave per SIMD starts its MFMAs at once
    // while the other issues the DMA, instead of both issuing before either computes
    // (4-6 % per launch, profiles/r04_dma_split_ab.txt).
    const bool dma_wave = wave < 4;
    int pk[2][G::PPW];
#pragma unroll
    for (int v = 0; v < 2; v++)
#pragma unroll
    for (int j = 0; j < G::PPW; j++) {
        const int vw = (wave & 3) + 4 * v;
        const int s = (j * G::NW + vw) * 64 + lane;
        int kind = 0, off = 0, nb = 0, hy = 0;
        if (s < G::HT) {
            const int hp = s / 3, q = s - hp * 3;
            if (hp > 0 && q < 2) {
                const int t = hp - 1;
                nb = t / G::CS;
                const int rr = t - nb * G::CS;
                hy = rr / G::RS;
                const int hx = rr - hy * G::RS;
                if (hx < W) {
                    kind = 1;
                    off = ((nb * H + hy - 1) * W + hx) * CIN + q * 8;
                }
            }
        } else if (s < G::HT + G::WT) {  // the weight image is in slot order: 1 KB contiguous per piece
            kind = 2;
            off = (s - G::HT) * 8;
        }
        pk[v][j] = (kind << 29) | (nb << 24) | (hy << 19) | off;
    }
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots16 - 1)) * 8;

    // tile -> (spatial tile, cout block), XCD-major: tiles t and t + 8 (same XCD under the
    // round-robin dispatch) are the two cout blocks of one spatial tile
    auto tile_of = [&](int tile, int& n0, int& ho0, int& cb) {
        const int j = tile >> 3;
        cb = j % p.ncb;
        const int sp = (j / p.ncb) * 8 + (tile & 7);
        n0 = (sp / tiles_h) * NB;
        ho0 = (sp - (sp / tiles_h) * tiles_h) * TH;
    };
    auto issue = [&](int item, int buf) {
        const int tile = blockIdx.x + (item / G::NCH) * gridDim.x, chunk = item % G::NCH;
        int n0, ho0, cb;
        tile_of(tile, n0, ho0, cb);
        const uint16_t* xb = p.x + ((long)(n0 * H + ho0) * W) * CIN + chunk * 16;
        const uint16_t* wb = p.w + (long)(cb * G::NCH + chunk) * G::WT * 8;
        uint8_t* dst = lds + buf * G::BUF;
        if (!dma_wave) return;
#pragma unroll
        for (int v = 0; v < 2; v++)
#pragma unroll
        for (int j = 0; j < G::PPW; j++) {
            const int vw = (wave & 3) + 4 * v;
            const int g = pk[v][j], kind = g >> 29, nb = (g >> 24) & 31, hy = (g >> 19) & 31, off = g & 0x7ffff;
            const bool in = kind == 1 && (unsigned)(ho0 + hy - 1) < (unsigned)H && n0 + nb < p.N;
            const uint16_t* src = kind == 2 ? wb + off : in ? xb + off : zl;
            // pieces wholly past the item's slots (6 of 64 on the 128-ch plane) are not issued
            if (j < G::PPW - 1 || (j * G::NW + vw) * 64 < G::HT + G::WT)
                glds16(src, dst + (j * G::NW + vw) * 1024);
        }
    };

    // ---- fragment bases (bytes) and output geometry
    const auto& map = kHMap<H, W, TH, NB>;
    int bv[G::NT], eoff[G::NT];  // output pixel (crop nb = eoff / (H * W)) from the tile's (n0, ho0, 0)
#pragma unroll
    for (int t = 0; t < G::NT; t++) {
        const int pp = map.pix[((pg * G::NT + t) * 2 + lane_grp(r32)) * 16 + lane_pos(r32)];
        const int nb = pp / (TH * W), rem = pp - nb * (TH * W);
        const int ty = rem / W, x = rem - (rem / W) * W;
        bv[t] = ((nb * G::CS + ty * G::RS + x) * 3 + h) * 16;
        eoff[t] = (nb * H + ty) * W + x;
    }
    const int av = (G::HT + h * BM + mg * 64 + r32) * 16;  // + a * 512 + tap * 2 * BM * 16

    const int n_items = ((p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) * G::NCH;
    // the workgroup's cout block is fixed (launcher: grid % (8 * ncb) == 0 or one tile each):
    // its folded-BN biases sit in LDS past the ring (registers would spill with the residual)
    {
        int cb0, n00, ho00;
        tile_of(blockIdx.x, n00, ho00, cb0);
        if (tid < BM) reinterpret_cast<float*>(lds + G::BIAS_OFF)[tid] = p.bias[cb0 * BM + tid];
    }
    const int bias_lds = G::BIAS_OFF + (mg * 64 + 16 * h) * 4;  // + a * 128
    issue(0, 0);
    f32x16 acc[G::NA][G::NT];
    for (int k = 0; k < n_items; k++) {
        const int buf = k & 1, chunk = k % G::NCH;
        const bool first = chunk == 0, last = chunk == G::NCH - 1;
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
        if (first) {
#pragma unroll
            for (int a = 0; a < G::NA; a++) {
                const f32x16 b = *reinterpret_cast<const f32x16*>(lds + bias_lds + a * 128);
#pragma unroll
                for (int t = 0; t < G::NT; t++) acc[a][t] = b;
            }
        }
        const long pix0 = (long)(n0 * H + ho0) * W;
        const int cob = cb * BM + mg * 64 + 16 * h;  // + a * 32
        uint4 rv[G::NA][G::NT][2];
        if (RES && last) {
#pragma unroll
            for (int a = 0; a < G::NA; a++)
#pragma unroll
                for (int t = 0; t < G::NT; t++) {
                    const bool ok = n0 + eoff[t] / (H * W) < p.N;
                    const uint16_t* rs = ok ? p.res + (pix0 + eoff[t]) * p.Cout + cob + a * 32 : p.zero + lane * 16;
                    rv[a][t][0] = *reinterpret_cast<const uint4*>(rs);
                    rv[a][t][1] = *reinterpret_cast<const uint4*>(rs + 8);
                }
        }
        asm volatile("" ::: "memory");
        const bool more = k + 1 < n_items;
        issue(more ? k + 1 : k, buf ^ 1);  // unconditional: see tconv.hip
        asm volatile("" ::: "memory");

        const int boff = buf * G::BUF;
        int bva[G::NT];
#pragma unroll
        for (int t = 0; t < G::NT; t++) bva[t] = bv[t] + boff;
        const int ava = av + boff;
        constexpr int NBF = 2;
        bf16x8 fa[NBF][G::NA], fb[NBF][G::NT];
        auto load = [&](int tap, bf16x8 (&a)[G::NA], bf16x8 (&b)[G::NT]) {
            const int dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int i = 0; i < G::NA; i++)
                a[i] = *reinterpret_cast<const bf16x8*>(lds + ava + (tap * 2 * BM + i * 32) * 16);
#pragma unroll
            for (int t = 0; t < G::NT; t++)
                b[t] = *reinterpret_cast<const bf16x8*>(lds + bva[t] + (dy * G::RS + dx) * 3 * 16);
        };
        load(0, fa[0], fb[0]);
#pragma unroll
        for (int tap = 0; tap < 9; tap++) {
            const int cur = tap & 1;
            if (tap + 1 < 9) load(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int a = 0; a < G::NA; a++)
#pragma unroll
                for (int t = 0; t < G::NT; t++)
                    acc[a][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][a], fb[cur][t], acc[a][t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        if (last) {
            // the residual loads precede this item's DMA pieces (PPW, or PPW - 1 on the waves whose
            // last piece is past the item): wait for all but PPW - 1 of them
            if (RES) {
                if (dma_wave)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::PPW - 2) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
#pragma unroll
            for (int a = 0; a < G::NA; a++)
#pragma unroll
                for (int t = 0; t < G::NT; t++) {
                    const bool ok = n0 + eoff[t] / (H * W) < p.N;
                    uint16_t* yrow = ok ? p.y + (pix0 + eoff[t]) * p.Cout + cob + a * 32 : p.sink + lane * 16;
                    uint32_t o[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        float v0 = acc[a][t][2 * e], v1 = acc[a][t][2 * e + 1];
                        if (RES) {
                            const uint4 rr = rv[a][t][e >> 2];
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

int g_t16_cus = 0;
uint16_t* g_t16_sink = nullptr;

template <int CIN, int H, int W, int TH, int NB, int BM, bool RES>
void launch_k16(const T16Params& p, int grid, hipStream_t s) {
    using G = T16Cfg<CIN, H, W, TH, NB, BM>;
    auto kern = tconv16_kernel<CIN, H, W, TH, NB, BM, RES>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT_THREADS), G::LDS, s, p);
}

template <int CIN, int H, int W, int TH, int NB, int BM>
void launch_t16(const ConvLaunch& c, hipStream_t s) {
    static_assert(HMap<H, W, TH, NB>().balanced(), "halo residues must be balanced for the lane map");
    if (g_t16_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_t16_cus, hipDeviceAttributeMultiprocessorCount, dev));
        MVP_HIP(hipMalloc(&g_t16_sink, 64 * 32));
    }
    MVP_REQUIRE(c.Cout % BM == 0, "tconv16: Cout %d not a multiple of %d", c.Cout, BM);
    const int ncb = c.Cout / BM;
    const long n_sp = (long)((c.N + NB - 1) / NB) * (H / TH);
    const long n_sp8 = (n_sp + 7) / 8 * 8;  // XCD-major tile order: spatial tiles in groups of 8
    const long tiles = n_sp8 * ncb;
    MVP_REQUIRE(tiles < (1L << 30), "tconv16: too many tiles");
    int grid = (int)std::min<long>(tiles, g_t16_cus);
    if (grid < tiles) grid -= grid % (8 * ncb);  // fixed cout block per workgroup
    MVP_REQUIRE(grid > 0, "tconv16: %d CUs", g_t16_cus);
    T16Params p{c.x, c.w_img, c.bias, c.res, c.y, conv_zero_region(), g_t16_sink, c.N, c.Cout, (int)tiles, ncb};
    if (c.res)
        launch_k16<CIN, H, W, TH, NB, BM, true>(p, grid, s);
    else
        launch_k16<CIN, H, W, TH, NB, BM, false>(p, grid, s);
}

// Weight image: for each (128-cout block cb, 16-cin chunk) the item's LDS weight slots in
// order, slot ws = (tap * 2 + q) * 128 + co holding w[cs][tap][16 chunk + 8 q .. + 8] with cs
// the permuted cout of A row co (row_cout within each 32-row group).
__global__ void tconv16_pack_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ img, int cin, int cout) {
    constexpr int BM = 128, WT = 9 * 2 * BM;
    const int nch = cin / 16;
    const long n = (long)(cout / BM) * nch * WT;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int ws = (int)(i % WT);
        const long cc = i / WT;
        const int chunk = (int)(cc % nch), cb = (int)(cc / nch);
        const int tq = ws / BM, co = ws - tq * BM;
        const int cs = cb * BM + ((co & ~31) | row_cout(co & 31));
        const uint16_t* src = w + ((long)cs * 9 + (tq >> 1)) * cin + chunk * 16 + (tq & 1) * 8;
        *reinterpret_cast<uint4*>(img + i * 8) = *reinterpret_cast<const uint4*>(src);
    }
}

bool t16_plane(int cin, int cout, int h, int w) {
    return (cin == 128 && cout == 128 && h == 16 && w == 12) || (cin == 256 && cout % 128 == 0 && h == 8 && w == 6);
}

}  // namespace

long tconv16_image_elems(int cin, int cout, int h, int w, int ks, int stride) {
    // stride 1: this file's planes; stride 2: s2conv.hip's streamed-weight planes (same
    // [tap][plane][128 couts] item image: transition2 / 3 and the fuse-layer chains' last convs)
    const bool s1 = stride == 1 && t16_plane(cin, cout, h, w);
    const bool s2 = stride == 2 && ((h == 32 && w == 24 && cout == 128 && cin == 64) ||
                                    (h == 16 && w == 12 && cout % 128 == 0 && (cin == 32 || cin == 64 || cin == 128)));
    return (ks == 3 && (s1 || s2)) ? (long)cout * 9 * cin : 0;
}

void tconv16_pack_weights(const uint16_t* w, uint16_t* img, int cin, int cout, hipStream_t s) {
    MVP_REQUIRE(cin % 16 == 0 && cout % 128 == 0, "tconv16_pack_weights: cin %d, cout %d", cin, cout);
    hipLaunchKernelGGL(tconv16_pack_kernel, dim3(256), dim3(256), 0, s, w, img, cin, cout);
    MVP_HIP(hipGetLastError());
}

bool launch_tconv16(const ConvLaunch& c, hipStream_t s) {
    if (!c.w_img || c.ks != 3 || c.stride != 1 || c.out_f32_nchw || !c.relu || c.x_stride || c.y_stride ||
        c.r_stride || c.x2)
        return false;
    const char* e = getenv("MVPOSE_TCONV16");  // A/B and tests: 0 = tconv.hip's 64-cout tiles
    if (e && e[0] == '0') return false;
    if (c.Cin == 128 && c.Cout == 128 && c.H == 16 && c.W == 12) {
        launch_t16<128, 16, 12, 16, 2, 128>(c, s);
        return true;
    }
    if (c.Cin == 256 && c.Cout % 128 == 0 && c.H == 8 && c.W == 6) {
        launch_t16<256, 8, 6, 8, 8, 128>(c, s);
        return true;
    }
    return false;
}

}  // namespace mvp
