// Fused HRNet stem for gfx950: conv1 (3x3/s2, 4 -> 64, BN + ReLU) and conv2
// (3x3/s2, 64 -> 64, BN + ReLU) in one launch, on 32x32x16 MFMAs:
//   y = relu(conv2(relu(conv1(x) + b1), w2) + b2),  x [N][256][192][4] -> y [N][64][48][64]
// Unfused, conv1 wrote its 128x96x64 output (1.57 MB per crop, 1.6 GB per 1024
// crops) and conv2 read it back; here conv1's output for the rows one tile of
// conv2 needs lives only in LDS (bf16, as the unfused graph rounds it), so HBM
// sees the 4-channel input (with a row halo) and conv2's output only.
//
// Tile = TR = 2 output rows (x 48 columns) of one crop, persistent workgroups of
// 8 waves (one per CU):
//   input rows   4r0-3 .. 4r0+7 (11 rows x 196 pixels incl. a 2-pixel zero border)
//                by LDS-DMA, issued under the previous tile's conv2
//   conv1        5 rows x 96 columns (rows 2r0-1 .. 2r0+3; row -1 = conv2's zero
//                padding), K = 9 taps x 4 ch padded to 48 (3 k-steps), A fragments
//                (stem weights, bf16) in registers, B = two 8-B taps per lane
//   intermediate split by column phase so every conv2 tap is [base + immediate]:
//                O[r][j] = conv1 column 2j-1 (O[r][0] = column -1 = zero pad),
//                E[r][j] = conv1 column 2j; output column c reads O[c], E[c], O[c+1]
//                (taps dx = 0, 1, 2) of rows 2lr+dy.  Chunk-major planes of 8 channels.
//   conv2        96 output pixels = 3 fragments x 2 cout groups = 6 wave units of
//                36 k-steps (9 taps x 4), weights resident in LDS ([tap][q][row],
//                rows = permuted couts so a lane owns 16 consecutive couts)
// K order differs from the unfused kernels', so results agree with them to f32
// summation-order rounding, not bit for bit.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;

struct S2 {
    static constexpr int H = 256, W = 192, W1 = 96, H2 = 64, W2 = 48;
    static constexpr int TR = 2;                       // conv2 output rows per tile
    static constexpr int NW = 8, NTH = NW * 64;
    static constexpr int R1 = 2 * TR + 1;              // conv1 rows per tile
    static constexpr int RX = 4 * TR + 3;              // input rows per tile
    static constexpr int XP = W + 4;                   // staged input row (pixels): 2 zero pixels each side
    static constexpr int XPIECES = XP * 8 / 16;        // 16-B pieces per staged row (98)
    static constexpr int XN = RX * XPIECES;            // pieces per tile (1078)
    static constexpr int XINSTR = (XN + 63) / 64;      // wave DMA instructions per tile (17)
    static constexpr int RS = W2 + 1;                  // intermediate row pitch (slots)
    static constexpr int PH = R1 * RS;                 // one phase image (slots)
    static constexpr int PLANE = 2 * PH;               // O then E image of one 8-channel plane
    static constexpr int WSLOTS = 9 * 8 * 64;          // conv2 weight slots
    static constexpr int W2OFF = 0;
    static constexpr int MOFF = W2OFF + WSLOTS * 16;
    static constexpr int XOFF = MOFF + 8 * PLANE * 16;
    static constexpr int BOFF = XOFF + XINSTR * 1024;
    static constexpr int LDS = BOFF + 2 * 64 * 4;
    static constexpr int F1 = R1 * W1 / 32;            // conv1 fragments (15)
    static constexpr int F2 = TR * W2 / 32;            // conv2 fragments (3)
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(R1 * W1 % 32 == 0 && TR * W2 % 32 == 0 && W1 % 16 == 0 && W2 % 16 == 0, "fragments");
    static_assert((6 * PLANE + 2 * RS + PH + 1) * 16 < 65536, "ds_read offset range (conv2 B)");
    static_assert((4 * 8 + 6) * 64 * 16 < 65536, "ds_read offset range (conv2 A, split at tap 4)");
};

struct StemParams {
    const uint16_t* x;
    const float* w1;    // [64][3][3][4] f32 (BN folded)
    const float* b1;    // [64]
    const uint16_t* w2; // [64][3][3][64] bf16 (BN folded)
    const float* b2;    // [64]
    uint16_t* y;
    const uint16_t* zero;
    int N, n_tiles;
};

__global__ __launch_bounds__(512, 1) void stem2_tile_kernel(StemParams p) {
    using G = S2;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = G::H2 / G::TR;
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    // ---- conv2 weights resident: slot s = (tap * 8 + q) * 64 + row, row = permuted cout
    for (int s0 = wave * 64; s0 < G::WSLOTS; s0 += G::NTH) {
        const int s = s0 + lane, row = s & 63, q = (s >> 6) & 7, tap = s >> 9;
        const int co = (row & ~31) | row_cout(row & 31);
        glds16(p.w2 + (co * 9 + tap) * 64 + q * 8, lds + G::W2OFF + s0 * 16);
    }
    // ---- the intermediate starts zero (O[r][0] = column -1 stays zero for the launch)
    for (int i = tid; i < 8 * G::PLANE; i += G::NTH)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    float* sbias = reinterpret_cast<float*>(lds + G::BOFF);
    if (tid < 64) sbias[tid] = p.b1[tid];
    else if (tid < 128) sbias[tid] = p.b2[tid - 64];

    // ---- conv1 A fragments (bf16, registers): this wave's cout group mg1, 3 k-steps;
    // k-step s, half h covers taps 4s + 2h and 4s + 2h + 1 (x 4 channels); taps >= 9 zero
    const int mg1 = wave & 1;
    bf16x8 a1[3];
    {
        const int co = mg1 * 32 + row_cout(r32);
#pragma unroll
        for (int s = 0; s < 3; s++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int tap = 4 * s + 2 * h + (j >> 2), ch = j & 3;
                a1[s][j] = (__bf16)(tap < 9 ? p.w1[(co * 9 + tap) * 4 + ch] : 0.f);
            }
    }
    // per-lane tap offsets (bytes) into the staged input, relative to the pixel's (row 2cr, px 2cc + 1)
    int toff[3][2];
#pragma unroll
    for (int s = 0; s < 3; s++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int tap = 4 * s + 2 * h + j;
            toff[s][j] = tap < 9 ? ((tap / 3) * G::XP + tap % 3) * 8 : -1;  // -1: zero tap (K padding)
        }

    // ---- input DMA geometry: instruction j of a tile = pieces 64j .. 64j + 63 (row-major
    // [row][piece]); this wave issues j = wave, wave + 8, wave + 16
    constexpr int XJ = (G::XINSTR + G::NW - 1) / G::NW;
    int xg[XJ];  // (row + 1) << 8 | piece, 0 = zero piece
#pragma unroll
    for (int m = 0; m < XJ; m++) {
        const int i = (wave + m * G::NW) * 64 + lane;
        const int row = i / G::XPIECES, k = i - row * G::XPIECES;
        xg[m] = (i < G::XN && k >= 1 && k <= G::W / 2) ? ((row + 1) << 8) | k : 0;
    }
    auto issue = [&](int item) {
        const int tile = blockIdx.x + item * gridDim.x;
        const int n = tile / tiles_h, r0 = (tile - n * tiles_h) * G::TR;
        const uint16_t* xb = p.x + (long)n * G::H * G::W * 4;
#pragma unroll
        for (int m = 0; m < XJ; m++) {
            const int j = wave + m * G::NW;
            if (j < G::XINSTR) {
                const int g = xg[m], row = (g >> 8) - 1, k = g & 255;
                const int gr = 4 * r0 - 3 + row;
                const bool in = g != 0 && (unsigned)gr < (unsigned)G::H;
                glds16(in ? xb + ((long)gr * G::W + 2 * (k - 1)) * 4 : zl, lds + G::XOFF + j * 1024);
            }
        }
    };

    // ---- conv1 fragments of this wave: f = (wave >> 1) + 4i
    const int nf1 = ((G::F1 - (wave >> 1)) + 3) / 4;  // 4 or 3
    int xb1[4], mw1[4], cr1[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int f = (wave >> 1) + 4 * i;
        if (f >= G::F1) f = 0;
        const int pp = frag_pixel<G::W1, G::R1, 1>(f, r32);
        const int cr = pp / G::W1, cc = pp - cr * G::W1;
        cr1[i] = cr;
        xb1[i] = G::XOFF + ((2 * cr) * G::XP + 2 * cc + 1) * 8;
        const int slot = (cc & 1) ? cr * G::RS + (cc + 1) / 2 : G::PH + cr * G::RS + cc / 2;
        mw1[i] = G::MOFF + ((mg1 * 4 + 2 * h) * G::PLANE + slot) * 16;
    }
    // ---- conv2 unit of this wave (waves 0..5): cout group mg2, fragment f2
    const bool has2 = wave < 2 * G::F2;
    const int mg2 = wave & 1, f2 = has2 ? (wave >> 1) : 0;
    int bv2, e2;
    {
        const int pp = frag_pixel<G::W2, G::TR, 1>(f2, r32);
        const int lr = pp / G::W2, c = pp - lr * G::W2;
        bv2 = G::MOFF + (h * G::PLANE + 2 * lr * G::RS + c) * 16;
        e2 = lr * G::W2 + c;
    }
    const int av2 = G::W2OFF + (h * 64 + mg2 * 32 + r32) * 16;
    auto bias16 = [&](int conv, int mg) {
        f32x16 v;
        const float4* b = reinterpret_cast<const float4*>(sbias + 64 * conv + mg * 32 + 16 * h);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float4 q = b[j];
            v[4 * j] = q.x;
            v[4 * j + 1] = q.y;
            v[4 * j + 2] = q.z;
            v[4 * j + 3] = q.w;
        }
        return v;
    };

    const int n_items = (p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    issue(0);
    for (int k = 0; k < n_items; k++) {
        // the tile's input has landed (younger: this wave's 2 conv2 stores of the previous tile)
        if (k == 0)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // + M zeroing, biases
        else if (!has2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();  // input visible; the previous tile's conv2 reads of M are done
        asm volatile("" ::: "memory");
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, r0 = (tile - n * tiles_h) * G::TR;

        // ---- conv1 -> intermediate (conv1 row -1 = conv2's zero padding)
        {
            const f32x16 b = bias16(0, mg1);
            f32x16 acc[4];
#pragma unroll
            for (int i = 0; i < 4; i++) acc[i] = b;
#pragma unroll
            for (int s = 0; s < 3; s++) {
                bf16x8 bf[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    union {
                        uint2 u[2];
                        bf16x8 v;
                    } t;
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const uint2 v = *reinterpret_cast<const uint2*>(lds + xb1[i] + max(toff[s][j], 0));
                        t.u[j] = toff[s][j] >= 0 ? v : uint2{0u, 0u};
                    }
                    bf[i] = t.v;
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (i < nf1) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[s], bf[i], acc[i], 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (i < nf1) {
                    const bool live = 2 * r0 - 1 + cr1[i] >= 0;
                    uint32_t o[8];
#pragma unroll
                    for (int e = 0; e < 8; e++)
                        o[e] = live ? pack_bf16x2(relu1(acc[i][2 * e]), relu1(acc[i][2 * e + 1])) : 0u;
                    *reinterpret_cast<uint4*>(lds + mw1[i]) = uint4{o[0], o[1], o[2], o[3]};
                    *reinterpret_cast<uint4*>(lds + mw1[i] + G::PLANE * 16) = uint4{o[4], o[5], o[6], o[7]};
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // intermediate complete, staged input free
        asm volatile("" ::: "memory");
        if (k + 1 < n_items) issue(k + 1);  // streams in under conv2
        asm volatile("" ::: "memory");

        // ---- conv2 + bias + ReLU -> 2 x 16-B stores (6 of the 8 waves)
        if (has2) {
            f32x16 acc = bias16(1, mg2);
            bf16x8 fa[2], fb[2];
            auto load = [&](int step, bf16x8& a, bf16x8& b) {
                const int tap = step >> 2, kq = step & 3, dy = tap / 3, dx = tap % 3;
                const int aoff = tap < 4 ? (tap * 8 + 2 * kq) * 64 * 16 : 32768 + ((tap - 4) * 8 + 2 * kq) * 64 * 16;
                a = *reinterpret_cast<const bf16x8*>(lds + av2 + aoff);
                const int boff = (kq * 2 * G::PLANE + dy * G::RS + (dx == 1 ? G::PH : dx == 2 ? 1 : 0)) * 16;
                b = *reinterpret_cast<const bf16x8*>(lds + bv2 + boff);
            };
            load(0, fa[0], fb[0]);
#pragma unroll
            for (int step = 0; step < 36; step++) {
                const int cur = step & 1;
                if (step + 1 < 36) load(step + 1, fa[cur ^ 1], fb[cur ^ 1]);
                __builtin_amdgcn_sched_barrier(0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur], acc, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) o[e] = pack_bf16x2(relu1(acc[2 * e]), relu1(acc[2 * e + 1]));
            uint16_t* yp = p.y + (((long)n * G::H2 + r0) * G::W2 + e2) * 64 + mg2 * 32 + 16 * h;
            *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ------------------------------------------------------------------ streaming version
// Same arithmetic as stem2_tile_kernel (conv1: 3 k-steps of taps 4s + 2h + j; conv2: 36
// k-steps (tap, 16-channel quarter) from the bias), hence bit-identical to it, but:
//  * each workgroup walks whole crops top to bottom in strips of 2 conv2 rows; conv1's rows
//    go into a 10-row LDS ring (virtual row v = crop * 129 + conv1 row + 1, row -1 = conv2's
//    zero padding), so no conv1 row is computed twice (the tile kernel recomputed 1 of 5);
//  * warp-specialised phases, one barrier each: waves 4-7 run conv1 of strip g (4 new rows:
//    6 of the 12 fragments x one 32-cout group each), waves 0-3 conv2 of strip g-1 (32-pixel
//    x 32-cout units: two interleaved chains on waves 0-1, one on waves 2-3; the cout group's
//    36 A fragments resident in 144 VGPRs); in the tile kernel conv1 and conv2 were
//    barrier-separated and two of the four SIMDs ran half of conv2's units.  Measured
//    (profiles/r04_stem2_streaming_ab.txt): 6 conv2 + 2 conv1 waves left the conv1 waves
//    the critical path (their LDS-read latency), 4 + 4 runs 15 % under the tile kernel;
//  * the input rows of strip g+1 (9 rows, 14 KB) land by LDS-DMA into the second input
//    buffer under phase g.
// Ring layout [ring row][image O | E][plane (8 ch)][49 slots]: every conv2 tap is a per-row
// base register + an immediate below 11 KB.
struct S2S {
    static constexpr int H = 256, W = 192, H1 = 128, W1 = 96, H2 = 64, W2 = 48;
    static constexpr int STRIPS = H2 / 2;              // strips of 2 conv2 rows per crop
    static constexpr int VR = H1 + 1;                  // virtual conv1 rows per crop (row -1 = zero)
    static constexpr int NR = 10;                      // ring rows (widest live span: crop boundary)
    static constexpr int RS = W2 + 1;                  // slots per image row
    static constexpr int ROWB = 2 * 8 * RS * 16;       // bytes per ring row (O and E, 8 planes)
    static constexpr int XP = W + 4;                   // staged input row: 2 zero pixels each side
    static constexpr int XPIECES = XP * 8 / 16;        // 98
    static constexpr int XROWS = 9;                    // input rows per strip
    static constexpr int XN = XROWS * XPIECES;         // 882 pieces
    static constexpr int XINSTR = (XN + 63) / 64;      // 14 wave DMA instructions
    static constexpr int MOFF = 0;
    static constexpr int XOFF = MOFF + NR * ROWB;      // 2 input buffers
    static constexpr int XBYTES = XINSTR * 1024;
    static constexpr int BOFF = XOFF + 2 * XBYTES;
    static constexpr int LDS = BOFF + 2 * 64 * 4;
    static constexpr int F1 = 4 * W1 / 32;             // 12 conv1 fragments per strip
    static constexpr int F2 = 2 * W2 / 32;             // 3 conv2 fragments per strip
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert((6 * RS + 8 * RS) * 16 < 65536, "ds_read offset range (conv2 B)");
    static_assert(XINSTR <= 4 * 4, "DMA: the 4 conv1 waves, up to 4 pieces each");
    static_assert(F2 == 3 && F1 == 2 * 2 * 3, "roles: conv2 fragments 0, 1 | 2; conv1 halves of 2 groups of 3");
};

__global__ __launch_bounds__(512, 1) void stem2_kernel(StemParams p) {
    using G = S2S;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nb = gridDim.x, b = blockIdx.x;
    const int crop0 = (int)(((long)p.N * b) / nb), crop1 = (int)(((long)p.N * (b + 1)) / nb);
    const int n_strips = (crop1 - crop0) * G::STRIPS;
    if (n_strips == 0) return;  // whole workgroup: uniform
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    // ---- the ring starts zero (O[r][0] = conv1 column -1 stays zero for the launch)
    for (int i = tid; i < G::NR * G::ROWB / 16; i += 512)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    float* sbias = reinterpret_cast<float*>(lds + G::BOFF);
    if (tid < 64) sbias[tid] = p.b1[tid];
    else if (tid < 128) sbias[tid] = p.b2[tid - 64];

    // ---- input DMA: instruction j of a strip = pieces 64j .. 64j + 63 ([row][piece]); the
    // conv1 waves issue all 14 (wave w: j = (w & 3) + 4m), the conv2 waves none, so each SIMD's
    // conv2 wave starts its MFMAs at once (same box: 425 -> 337 us; split over all 8 waves as
    // before, or all on the conv2 waves: 364 -- profiles/r04_dma_split_ab.txt)
    const bool dma_wave = wave >= 4;
    int xg[4];  // (row + 1) << 8 | piece, 0 = zero piece
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int i = ((wave & 3) + m * 4) * 64 + lane;
        const int row = i / G::XPIECES, k = i - row * G::XPIECES;
        xg[m] = (i < G::XN && k >= 1 && k <= G::W / 2) ? ((row + 1) << 8) | k : 0;
    }
    auto issue = [&](int g) {  // strip g's 9 input rows -> buffer g & 1
        const int n = crop0 + g / G::STRIPS, s = g % G::STRIPS;
        const uint16_t* xb = p.x + (long)n * G::H * G::W * 4;
        uint8_t* dst = lds + G::XOFF + (g & 1) * G::XBYTES;
        if (!dma_wave) return;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int j = (wave & 3) + m * 4;
            if (j < G::XINSTR) {
                const int gg = xg[m], row = (gg >> 8) - 1, k = gg & 255;
                const int gr = 8 * s - 1 + row;
                const bool in = gg != 0 && (unsigned)gr < (unsigned)G::H;
                glds16(in ? xb + ((long)gr * G::W + 2 * (k - 1)) * 4 : zl, dst + j * 1024);
            }
        }
    };
    auto ring = [](int v) { return (v % G::NR) * G::ROWB; };

    if (wave < 4) {
        // ================= conv2 waves: cout group mg2 = wave & 1; waves 0-1 fragments 0 and 1
        // (two interleaved chains), waves 2-3 fragment 2
        const int mg2 = wave & 1;
        bf16x8 wa[36];
        {
            const int co = mg2 * 32 + row_cout(r32);
#pragma unroll
            for (int st = 0; st < 36; st++) {
                const int tap = st >> 2, kq = st & 3;
                wa[st] = *reinterpret_cast<const bf16x8*>(p.w2 + (co * 9 + tap) * 64 + 16 * kq + 8 * h);
            }
        }
        auto run = [&](auto NUc) {
            constexpr int NU = decltype(NUc)::value;
            int lr[NU], c[NU];
#pragma unroll
            for (int u = 0; u < NU; u++) {
                const int f2 = NU == 2 ? u : 2;
                const int pp = frag_pixel<G::W2, 2, 1>(f2, r32);
                lr[u] = pp / G::W2;
                c[u] = pp - lr[u] * G::W2;
            }
            issue(0);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            for (int g = 0; g <= n_strips; g++) {
                if (g + 1 < n_strips) issue(g + 1);
                asm volatile("" ::: "memory");
                if (g >= 1) {
                    const int cl = (g - 1) / G::STRIPS, s = (g - 1) % G::STRIPS;
                    const int v0 = cl * G::VR + 4 * s;  // conv1 row 4s - 1
                    int bvd[NU][3];
#pragma unroll
                    for (int u = 0; u < NU; u++)
#pragma unroll
                        for (int dy = 0; dy < 3; dy++)
                            bvd[u][dy] = G::MOFF + ring(v0 + 2 * lr[u] + dy) + (h * G::RS + c[u]) * 16;
                    f32x16 acc[NU];
                    {
                        const float4* bb = reinterpret_cast<const float4*>(sbias + 64 + mg2 * 32 + 16 * h);
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const float4 q = bb[j];
                            acc[0][4 * j] = q.x;
                            acc[0][4 * j + 1] = q.y;
                            acc[0][4 * j + 2] = q.z;
                            acc[0][4 * j + 3] = q.w;
                        }
#pragma unroll
                        for (int u = 1; u < NU; u++) acc[u] = acc[0];
                    }
                    constexpr int kPF = NU == 2 ? 4 : 6;
                    bf16x8 fb[kPF + 1][NU];
                    auto load = [&](int st) {
                        const int tap = st >> 2, kq = st & 3, dy = tap / 3, dx = tap % 3;
#pragma unroll
                        for (int u = 0; u < NU; u++)
                            fb[st % (kPF + 1)][u] = *reinterpret_cast<const bf16x8*>(
                                lds + bvd[u][dy] + (2 * kq * G::RS + (dx == 1 ? 8 * G::RS : dx == 2 ? 1 : 0)) * 16);
                    };
#pragma unroll
                    for (int st = 0; st < kPF; st++) load(st);
#pragma unroll
                    for (int st = 0; st < 36; st++) {
                        if (st + kPF < 36) load(st + kPF);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < NU; u++)
                            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[st], fb[st % (kPF + 1)][u], acc[u], 0, 0, 0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int u = 0; u < NU; u++) {
                        uint32_t o[8];
#pragma unroll
                        for (int e = 0; e < 8; e++) o[e] = pack_bf16x2(relu1(acc[u][2 * e]), relu1(acc[u][2 * e + 1]));
                        uint16_t* yp = p.y + (((long)(crop0 + cl) * G::H2 + 2 * s + lr[u]) * G::W2 + c[u]) * 64 +
                                       mg2 * 32 + 16 * h;
                        *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
                        *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
                    }
                    // the next strip's input has landed (the 2 NU stores are younger)
                    if constexpr (NU == 2)
                        asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
                    else
                        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_s_barrier();
            }
        };
        if (wave < 2)
            run(std::integral_constant<int, 2>{});
        else
            run(std::integral_constant<int, 1>{});
    } else {
        // ================= conv1 waves: cout group mg1, fragments 6 half .. 6 half + 5 in 2 groups of 3
        const int mg1 = wave & 1, half = (wave - 4) >> 1;
        bf16x8 a1[3];
        {
            const int co = mg1 * 32 + row_cout(r32);
#pragma unroll
            for (int st = 0; st < 3; st++)
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int tap = 4 * st + 2 * h + (j >> 2), ch = j & 3;
                    a1[st][j] = (__bf16)(tap < 9 ? p.w1[(co * 9 + tap) * 4 + ch] : 0.f);
                }
        }
        int toff[3][2];
#pragma unroll
        for (int st = 0; st < 3; st++)
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int tap = 4 * st + 2 * h + j;
                toff[st][j] = tap < 9 ? ((tap / 3) * G::XP + tap % 3) * 8 : -1;
            }
        constexpr int NF = G::F1 / 2;
        int xo[NF], mo[NF], cro[NF];  // staged-input offset, ring slot offset, conv1 row in strip
#pragma unroll
        for (int f = 0; f < NF; f++) {
            const int pp = frag_pixel<G::W1, 4, 1>(half * NF + f, r32);
            const int cr = pp / G::W1, cc = pp - cr * G::W1;
            cro[f] = cr;
            xo[f] = ((2 * cr) * G::XP + 2 * cc + 1) * 8;
            const int img = (cc & 1) ? 0 : 1, j = (cc & 1) ? (cc + 1) / 2 : cc / 2;
            mo[f] = ((img * 8 + mg1 * 4 + 2 * h) * G::RS + j) * 16;
        }
        issue(0);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        for (int g = 0; g <= n_strips; g++) {
            if (g + 1 < n_strips) issue(g + 1);
            asm volatile("" ::: "memory");
            if (g < n_strips) {
                const int cl = g / G::STRIPS, s = g % G::STRIPS;
                const int v0 = cl * G::VR + 4 * s;
                const uint8_t* xb = lds + G::XOFF + (g & 1) * G::XBYTES;
                if (s == 0)  // conv1 row -1: conv2's zero padding
                    for (int i = (wave - 4) * 64 + lane; i < G::ROWB / 16; i += 256)
                        *reinterpret_cast<uint4*>(lds + G::MOFF + ring(v0) + i * 16) = uint4{0u, 0u, 0u, 0u};
                f32x16 bias;
                {
                    const float4* bb = reinterpret_cast<const float4*>(sbias + mg1 * 32 + 16 * h);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const float4 q = bb[j];
                        bias[4 * j] = q.x;
                        bias[4 * j + 1] = q.y;
                        bias[4 * j + 2] = q.z;
                        bias[4 * j + 3] = q.w;
                    }
                }
                // a group's 24 input reads are issued one group ahead (the MFMAs of a 3-step
                // group cover too little of the LDS latency on their own)
                uint2 raw[2][3][3][2];
                auto load_grp = [&](int grp, uint2 (&r)[3][3][2]) {
#pragma unroll
                    for (int st = 0; st < 3; st++)
#pragma unroll
                        for (int i = 0; i < 3; i++)
#pragma unroll
                            for (int j = 0; j < 2; j++)
                                r[st][i][j] = *reinterpret_cast<const uint2*>(xb + xo[grp * 3 + i] + max(toff[st][j], 0));
                };
                load_grp(0, raw[0]);
#pragma unroll
                for (int grp = 0; grp < 2; grp++) {
                    if (grp + 1 < 2) load_grp(grp + 1, raw[(grp + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);
                    f32x16 acc[3];
#pragma unroll
                    for (int i = 0; i < 3; i++) acc[i] = bias;
#pragma unroll
                    for (int st = 0; st < 3; st++) {
                        bf16x8 bf[3];
#pragma unroll
                        for (int i = 0; i < 3; i++) {
                            union {
                                uint2 u[2];
                                bf16x8 v;
                            } t;
#pragma unroll
                            for (int j = 0; j < 2; j++) t.u[j] = toff[st][j] >= 0 ? raw[grp & 1][st][i][j] : uint2{0u, 0u};
                            bf[i] = t.v;
                        }
#pragma unroll
                        for (int i = 0; i < 3; i++)
                            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[st], bf[i], acc[i], 0, 0, 0);
                    }
#pragma unroll
                    for (int i = 0; i < 3; i++) {
                        const int f = grp * 3 + i;
                        uint32_t o[8];
#pragma unroll
                        for (int e = 0; e < 8; e++) o[e] = pack_bf16x2(relu1(acc[i][2 * e]), relu1(acc[i][2 * e + 1]));
                        uint8_t* d = lds + G::MOFF + ring(v0 + 1 + cro[f]) + mo[f];
                        *reinterpret_cast<uint4*>(d) = uint4{o[0], o[1], o[2], o[3]};
                        *reinterpret_cast<uint4*>(d + G::RS * 16) = uint4{o[4], o[5], o[6], o[7]};
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
    }
}

int g_s2_cus = 0;

}  // namespace

bool stem2_supported(int H, int W, int cin2, int cout2) {
    const char* e = getenv("MVPOSE_NO_STEMFUSE");  // diagnostics/tests: run the two convs apart
    if (e && e[0] == '1') return false;
    return H == S2::H && W == S2::W && cin2 == 64 && cout2 == 64;
}

void launch_stem2(const uint16_t* x, const float* w1, const float* b1, const uint16_t* w2, const float* b2,
                  uint16_t* y, int N, int H, int W, hipStream_t s) {
    MVP_REQUIRE(H == S2::H && W == S2::W, "stem2: input %dx%d is not 256x192", H, W);
    if (N == 0) return;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)stem2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, S2S::LDS));
        attr = true;
    }
    if (g_s2_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_s2_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const char* e = getenv("MVPOSE_STEM2_TILE");  // tests: the tile kernel (bit-identical reference)
    if ((e && e[0] == '1') || !crop_ranges_balanced(N, g_s2_cus)) {  // + small / ragged batches
        static bool attr_t = false;
        if (!attr_t) {
            MVP_HIP(hipFuncSetAttribute((const void*)stem2_tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        S2::LDS));
            attr_t = true;
        }
        const long tiles = (long)N * (S2::H2 / S2::TR);
        MVP_REQUIRE(tiles < (1L << 30), "stem2: too many tiles");
        StemParams p{x, w1, b1, w2, b2, y, conv_zero_region(), N, (int)tiles};
        const int grid = (int)std::min<long>(tiles, g_s2_cus);
        hipLaunchKernelGGL(stem2_tile_kernel, dim3(grid), dim3(S2::NTH), S2::LDS, s, p);
        MVP_HIP(hipGetLastError());
        return;
    }
    MVP_REQUIRE(N < (1 << 24), "stem2: too many crops");
    StemParams p{x, w1, b1, w2, b2, y, conv_zero_region(), N, 0};
    const int grid = std::min(N, g_s2_cus);
    hipLaunchKernelGGL(stem2_kernel, dim3(grid), dim3(512), S2S::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
