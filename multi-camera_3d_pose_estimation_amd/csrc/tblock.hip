// Fused HRNet BasicBlock on 32 channels, 32x32x16 MFMAs (gfx950):
//   y = relu( conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x )
// for the 64x48 branch plane (32 of HRNet-W32's 120 BasicBlocks), one kernel:
// the intermediate never leaves LDS and the residual is read from the staged
// input halo, so HBM sees the input (with a 2-row halo) and the output only —
// the layer is HBM-bound at ~417 KB per crop and block.
//
// Same building blocks as tconv.hip: every fragment read is ds_read_b128 [base +
// immediate] on halo images stored chunk-major ([8-channel group q][slot]) with a
// row pitch of W+1 slots whose last slot is zero (+1 leading zero slot), so a
// tap (dy, dx) of output pixel (r, x) is slot base(r, x) + dy*(W+1) + dx with no
// border masking; A rows are a permutation of the 32 couts (row 8j+4h+i holds
// cout 16h+4j+i) so a lane owns 16 consecutive channels of its pixel.
//
// Persistent workgroups of 8 waves walk tiles of TH output rows of one crop:
//   input halo   (TH+4) rows x W, 4 planes; one buffer (its DMA for the next tile
//                streams under conv2) or a two-slot ring (DMA under the whole tile)
//   conv1        on TH+2 rows x W (fragments of 32 pixels) -> intermediate (bias,
//                ReLU, bf16; rows outside the image written as 0 = conv2's zero
//                padding)
//   conv2        TH rows x W -> + b2 + residual (the input halo's centre rows),
//                ReLU -> 2 x 16-B stores per fragment and lane
// Weights of both convs stay resident (36.9 KiB).  Deployed: TH = 16, one buffer
// (158.9 KiB LDS; fragments per SIMD per tile 13/13/13/12), one workgroup per CU,
// two waves per SIMD.
// K order (tap, cin) differs from conv_mfma_kernel's, so results agree with the
// two separate convs to f32 summation-order rounding, not bit for bit.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;


template <int W, int TH_, bool DB_, bool PAIR_ = false, bool SWZ_ = false>
struct TBCfg {
    static constexpr int NW = 8, NTH = NW * 64, TH = TH_;
    static constexpr bool DB = DB_;                       // double-buffered input halo
    // PAIR: the input halo's planes 2k, 2k+1 interleaved per pixel ([pair][pixel][2] slots):
    // a DMA instruction reads 32 contiguous bytes per pixel (half the cache lines of
    // plane-major) for 2-way bank conflicts on the conv1 fragment reads
    static constexpr bool PAIR = PAIR_;
    static constexpr int PX = PAIR ? 2 : 1;               // input-halo slots between pixels
    // SWZ (with PAIR): the two planes of pixel slot hs swap places when bit 3 of hs is set, so
    // 16 pixels distinct mod 16 hit 16 distinct 16-B bank positions (conflict-free conv1
    // fragment reads) at the price of per-tap address arithmetic
    static constexpr bool SWZ = SWZ_ && PAIR_;
    static constexpr int RS = W + 1;
    static constexpr int HSI = 1 + (TH + 4) * RS;        // input halo slots per plane
    static constexpr int HSM = 1 + (TH + 2) * RS;        // intermediate slots per plane
    static constexpr int XSLOTS = 4 * HSI;
    static constexpr int XPPW = (XSLOTS + 64 * NW - 1) / (64 * NW);  // DMA pieces per wave per tile
    static constexpr int XBYTES = XPPW * NW * 1024;      // one input-halo ring slot
    static constexpr int MOFF = (DB ? 2 : 1) * XBYTES, MBYTES = 4 * HSM * 16;
    static constexpr int WSL = 9 * 4 * 32;                // one conv's weight slots
    static constexpr int W1OFF = MOFF + MBYTES, W2OFF = W1OFF + WSL * 16;
    static constexpr int BOFF = W2OFF + WSL * 16;         // 2 x 32 f32 biases
    static constexpr int LDS = BOFF + 256;
    static constexpr int F1 = (TH + 2) * W / 32, F2 = TH * W / 32;  // fragments per tile
    static constexpr int MF1 = (F1 + NW - 1) / NW, MF2 = (F2 + NW - 1) / NW;  // max per wave
    static_assert((TH + 2) * W % 32 == 0 && TH * W % 32 == 0, "whole fragments");
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert((2 * HSI + 2 * RS + 2) * 16 < 65536, "ds_read offset range");
    static_assert(TH + 4 < 31 && (TH + 2) * W * 32 < (1 << 25), "packed DMA geometry");
    static_assert(2 * MF2 < 16 && XPPW < 64, "vmcnt range");
    static_assert(!SWZ || !DB, "the swizzled halo is single-buffered");
};

struct TBParams {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y;
    const uint16_t* zero;
    int N, H, n_tiles;
};

template <int W, int TH_, bool DB_, bool PAIR, bool SWZ = false>
__global__ __launch_bounds__(512, 1) void tblock32_kernel(TBParams p) {
    using G = TBCfg<W, TH_, DB_, PAIR, SWZ>;
    constexpr int TH = G::TH, RS = G::RS;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    const int H = p.H, tiles_h = H / TH;
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    // ---- weights of both convs, [tap][q][row] slots, rows = permuted couts
    for (int s0 = wave * 64; s0 < G::WSL; s0 += G::NTH) {
        const int sl = s0 + lane, r = sl & 31, tq = sl >> 5;
        const int off = (row_cout(r) * 9 + (tq >> 2)) * 32 + (tq & 3) * 8;
        glds16(p.w1 + off, lds + G::W1OFF + s0 * 16);
        glds16(p.w2 + off, lds + G::W2OFF + s0 * 16);
    }
    // ---- the intermediate's pad / leading slots stay zero for the launch
    for (int i = tid; i < G::MBYTES / 16; i += G::NTH)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};

    // ---- per-lane DMA geometry of this wave's input-halo pieces, one register each:
    // (element offset + 8192) << 5 | (halo row + 1), 0 for zero / padding slots
    int pk[G::XPPW];
#pragma unroll
    for (int j = 0; j < G::XPPW; j++) {
        const int s = (j * G::NW + wave) * 64 + lane;
        int g = -1, off = 0;
        if (s < G::XSLOTS) {
            const int hs = PAIR ? (s % (2 * G::HSI)) >> 1 : s - (s / G::HSI) * G::HSI;
            const int q = PAIR ? (s / (2 * G::HSI)) * 2 + ((s & 1) ^ (G::SWZ ? (hs >> 3) & 1 : 0)) : s / G::HSI;
            if (hs > 0) {
                const int t = hs - 1, hy = t / RS, hx = t - (t / RS) * RS;
                if (hx < W) {
                    g = hy;
                    off = ((hy - 2) * W + hx) * 32 + q * 8;  // from the tile's (row ho0, col 0)
                }
            }
        }
        pk[j] = g < 0 ? 0 : ((off + 8192) << 5) | (g + 1);
    }
    auto issue = [&](int k, int buf) {
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, ho0 = (tile - n * tiles_h) * TH;
        const uint16_t* xb = p.x + ((long)n * H + ho0) * W * 32;
#pragma unroll
        for (int j = 0; j < G::XPPW; j++) {
            const int g = pk[j], hy1 = g & 31;
            const bool in = hy1 != 0 && (unsigned)(ho0 + hy1 - 3) < (unsigned)H;
            glds16(in ? xb + ((g >> 5) - 8192) : zl, lds + buf * G::XBYTES + (j * G::NW + wave) * 1024);
        }
    };

    // ---- fragment geometry.  conv1 fragments f = wave + 8i (i < nf1), conv2 f = wave + 8i (i < nf2)
    const int nf1 = (G::F1 - wave + G::NW - 1) / G::NW;  // MF1 or MF1 - 1
    const int nf2 = (G::F2 - wave + G::NW - 1) / G::NW;  // MF2 or MF2 - 1
    const int av1 = G::W1OFF + (h * 32 + r32) * 16, av2 = G::W2OFF + (h * 32 + r32) * 16;
    int b1v[G::MF1], m1w[G::MF1], b2v[G::MF2], r2v[G::MF2], e2[G::MF2];
#pragma unroll
    for (int i = 0; i < G::MF1; i++) {
        int pp = frag_pixel<W, TH, 1>(wave + 8 * i, r32);
        if (pp >= (TH + 2) * W) pp = 0;  // unused slot
        const int r = pp / W, x = pp - (pp / W) * W;
        b1v[i] = (PAIR ? h + (r * RS + x) * 2 : h * G::HSI + r * RS + x) * 16;  // input halo, tap (0,0)
        m1w[i] = G::MOFF + (2 * h * G::HSM + 1 + r * RS + x) * 16;  // intermediate slot, plane 2h
    }
#pragma unroll
    for (int i = 0; i < G::MF2; i++) {
        int pp = frag_pixel<W, TH, 1>(wave + 8 * i, r32);
        if (pp >= TH * W) pp = 0;
        const int r = pp / W, x = pp - (pp / W) * W;
        b2v[i] = G::MOFF + (h * G::HSM + r * RS + x) * 16;              // intermediate, tap (0,0)
        // residual: input (r+2, x), planes 2h (first 16 B) and 2h+1 (second, + r2s)
        const int hr = 1 + (r + 2) * RS + x;
        r2v[i] = (2 * h * G::HSI + hr * G::PX + (G::SWZ ? (hr >> 3) & 1 : 0)) * 16;
        e2[i] = r * W + x;
    }
    // folded-BN biases in LDS (visible after the first tile's barrier): registers are the scarce resource
    float* sbias = reinterpret_cast<float*>(lds + G::BOFF);
    if (tid < 32) sbias[tid] = p.b1[tid];
    else if (tid < 64) sbias[tid] = p.b2[tid - 32];
    auto binit = [&](int conv2) {  // the lane's 16 couts 16h .. 16h+15
        f32x16 v;
        const float4* b = reinterpret_cast<const float4*>(sbias + 32 * conv2 + 16 * h);
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

    // one conv over NF fragments: 9 taps x 2 k-steps, fragments of step s+1 read before step s
    auto conv = [&](auto nf_tag, int av, const int* bv, int hs, auto px_tag, f32x16* acc) {
        constexpr int PXS = decltype(px_tag)::value;  // slots between pixels of this image
        constexpr int NF = decltype(nf_tag)::value;
        bf16x8 fa[2], fb[2][NF];
        auto load = [&](int step, bf16x8& a, bf16x8 (&b)[NF]) {
            const int tap = step >> 1, ks = step & 1, dy = tap / 3, dx = tap % 3;
            a = *reinterpret_cast<const bf16x8*>(lds + av + (tap * 4 + ks * 2) * 32 * 16);
#pragma unroll
            for (int t = 0; t < NF; t++) {
                if constexpr (G::SWZ && PXS == 2) {
                    int bt = bv[t];
                    asm volatile("" : "+v"(bt));  // per-step address math: 36 hoisted tap addresses spill
                    const int a = bt + (dy * RS + dx) * 32;  // (2*slot + h) * 16, unswizzled
                    b[t] = *reinterpret_cast<const bf16x8*>(lds + (a ^ ((a >> 4) & 16)) + ks * 2 * hs * 16);
                } else {
                    b[t] = *reinterpret_cast<const bf16x8*>(lds + bv[t] + (ks * 2 * hs + (dy * RS + dx) * PXS) * 16);
                }
            }
        };
        load(0, fa[0], fb[0]);
#pragma unroll
        for (int step = 0; step < 18; step++) {
            const int cur = step & 1;
            if (step + 1 < 18) load(step + 1, fa[cur ^ 1], fb[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < NF; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    const int n_items = (p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    issue(0, 0);
    for (int k = 0; k < n_items; k++) {
        const int buf = k & 1;
        // the tile's input halo has landed (younger: the previous tile's 2*nf2 stores);
        // the barrier publishes it and retires every read of the other ring slot and of
        // the previous tile's intermediate
        if (k == 0)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (nf2 == G::MF2)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::MF2) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::MF2 - 2) : "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (G::DB && k + 1 < n_items) issue(k + 1, buf ^ 1);  // streams in under this whole tile
        asm volatile("" ::: "memory");
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, ho0 = (tile - n * tiles_h) * TH;
        const int xoff = G::DB ? buf * G::XBYTES : 0;

        // ---- conv1 -> intermediate (rows outside the image: zeros)
        {
            f32x16 acc[G::MF1];
            const f32x16 b = binit(0);
#pragma unroll
            for (int i = 0; i < G::MF1; i++) acc[i] = b;
            int bv[G::MF1];
#pragma unroll
            for (int i = 0; i < G::MF1; i++) bv[i] = b1v[i] + xoff;
            if (nf1 == G::MF1)
                conv(std::integral_constant<int, G::MF1>{}, av1, bv, G::HSI, std::integral_constant<int, G::PX>{}, acc);
            else
                conv(std::integral_constant<int, G::MF1 - 1>{}, av1, bv, G::HSI, std::integral_constant<int, G::PX>{},
                     acc);
#pragma unroll
            for (int i = 0; i < G::MF1; i++) {
                if (i < nf1) {
                    const int pp = frag_pixel<W, TH, 1>(wave + 8 * i, r32);
                    const int iy = ho0 - 1 + pp / W;
                    const bool live = (unsigned)iy < (unsigned)H;
                    uint32_t o[8];
#pragma unroll
                    for (int e = 0; e < 8; e++)
                        o[e] = live ? pack_bf16x2(relu1(acc[i][2 * e]), relu1(acc[i][2 * e + 1])) : 0u;
                    *reinterpret_cast<uint4*>(lds + m1w[i]) = uint4{o[0], o[1], o[2], o[3]};
                    *reinterpret_cast<uint4*>(lds + m1w[i] + G::HSM * 16) = uint4{o[4], o[5], o[6], o[7]};
                }
            }
        }
        // single buffer: the residual leaves the input halo before the next tile's DMA
        uint4 rv[G::DB ? 1 : G::MF2][2];
        if (!G::DB) {
#pragma unroll
            for (int i = 0; i < (G::DB ? 1 : G::MF2); i++) {
                rv[i][0] = *reinterpret_cast<const uint4*>(lds + r2v[i]);
                rv[i][1] = *reinterpret_cast<const uint4*>(lds + (G::SWZ ? r2v[i] ^ 16 : r2v[i] + (PAIR ? 1 : G::HSI) * 16));
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // intermediate complete (and, single buffer, the input halo free)
        asm volatile("" ::: "memory");
        if (!G::DB && k + 1 < n_items) issue(k + 1, 0);  // streams in under conv2
        asm volatile("" ::: "memory");

        // ---- conv2 + bias + residual (input halo, still resident) + ReLU -> 2 x 16-B stores
        {
            f32x16 acc[G::MF2];
            const f32x16 b = binit(1);
#pragma unroll
            for (int i = 0; i < G::MF2; i++) acc[i] = b;
            if (nf2 == G::MF2)
                conv(std::integral_constant<int, G::MF2>{}, av2, b2v, G::HSM, std::integral_constant<int, 1>{}, acc);
            else
                conv(std::integral_constant<int, G::MF2 - 1>{}, av2, b2v, G::HSM, std::integral_constant<int, 1>{},
                     acc);
            const long pix0 = ((long)n * H + ho0) * W;
#pragma unroll
            for (int i = 0; i < G::MF2; i++) {
                if (i < nf2) {
                    uint4 ra, rb;
                    if (G::DB) {
                        ra = *reinterpret_cast<const uint4*>(lds + xoff + r2v[i]);
                        rb = *reinterpret_cast<const uint4*>(lds + xoff + r2v[i] + (PAIR ? 1 : G::HSI) * 16);
                    } else {
                        ra = rv[G::DB ? 0 : i][0];
                        rb = rv[G::DB ? 0 : i][1];
                    }
                    uint32_t o[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const uint4 rr = e < 4 ? ra : rb;
                        const uint32_t u = (e & 3) == 0 ? rr.x : (e & 3) == 1 ? rr.y : (e & 3) == 2 ? rr.z : rr.w;
                        o[e] = pack_bf16x2(relu1(acc[i][2 * e] + lo_bf16(u)), relu1(acc[i][2 * e + 1] + hi_bf16(u)));
                    }
                    uint16_t* yp = p.y + (pix0 + e2[i]) * 32 + 16 * h;
                    *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
                    *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int g_tb_cus = 0;

}  // namespace

bool launch_tblock32(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                     uint16_t* y, int N, int H, int W, hipStream_t s) {
    // TH = 16, single-buffered input halo: 82.7 us/conv at 1024 crops vs 91.0 for TH = 8
    // double-buffered (more conv1 recompute and input re-fetch) — tools/conv_bench.py
    using G = TBCfg<48, 16, false>;
    static_assert(TBCfg<48, 16, false, true>::LDS == G::LDS, "paired halo changes only the slot order");
    if (W != 48 || H % G::TH != 0) return false;
    const char* e = getenv("MVPOSE_NO_TBLOCK");  // diagnostics/tests: use basic_block_c32_kernel
    if (e && e[0] == '1') return false;
    if (N == 0) return true;
    // input halo planes 2k, 2k+1 interleaved per pixel (each DMA instruction touches half the
    // cache lines: +0.6 % frames/s over plane-major, round 2)
    auto kern = tblock32_kernel<48, 16, false, true>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (g_tb_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_tb_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long tiles = (long)N * (H / G::TH);
    MVP_REQUIRE(tiles < (1L << 30), "tblock: too many tiles");
    TBParams p{x, w1, b1, w2, b2, y, conv_zero_region(), N, H, (int)tiles};
    const int grid = (int)std::min<long>(tiles, g_tb_cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NTH), G::LDS, s, p);
    MVP_HIP(hipGetLastError());
    return true;
}

}  // namespace mvp
