// HRNet-W32 transition1 for gfx950: both 3x3 convs that read the layer1 output
// (64x48x256, 1.6 GB per 1024 crops) in ONE pass over it, on 32x32x16 MFMAs:
//   t0 = relu(conv3x3/s1(y, w0) + b0)   256 -> 32 ch @ 64x48   (transition1.0)
//   t1 = relu(conv3x3/s2(y, w1) + b1)   256 -> 64 ch @ 32x24   (transition1.1.0)
// Unfused, each conv streamed the whole 256-channel tensor (781 + 807 us per 1024
// crops, ~2 TB/s each).  Here a tile of TH = 16 rows of y (+ 1 halo row each side)
// arrives once, 16 channels at a time, and feeds both convs: t0's 16 output rows
// and t1's 8 output rows (t1 row r reads y rows 2r-1 .. 2r+1, inside the same halo).
//
// Work item = (tile, 16-channel chunk); per item one LDS-DMA ring slot holds the
// halo's two 8-channel planes (chunk-major [q][slot], row pitch W+1 with a zero pad
// slot, +1 leading zero slot: tap (dy, dx) of any output pixel is base + immediate,
// as in tconv.hip) and both convs' weight slices ([tap][q][row], rows = permuted
// couts so a lane owns 16 consecutive couts).  Two ring slots: item k+1 streams in
// while item k computes.  Waves 0-5 run t0 (4 fragments of 32 pixels each, one
// 32-cout group), waves 6-7 run t1 (6 fragments, one 32-cout group each); per item
// 36 / 54 MFMAs.  K order (chunk, tap, channel) differs from the separate kernels',
// so results agree with them to f32 summation-order rounding.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;

template <bool PM_>
struct T1C {
    static constexpr int H = 64, W = 48, C = 256, TH = 16;
    static constexpr int NW = 8, NTH = NW * 64;
    static constexpr int NCH = C / 16;                     // 16-channel items per tile
    static constexpr int RS = W + 1, HR = TH + 2;          // halo row pitch (pixels), rows
    static constexpr int HS = 1 + HR * RS;                 // halo pixels (incl. the leading zero)
    // PM (pixel-major halo): a pixel's two 16-B planes are slots 3p, 3p+1 (3p+2 a never-read
    // pad): a DMA instruction reads ~21 pixels x 32 contiguous bytes instead of 64 pixels x
    // 16 B (a third of the cache lines); the 48-B pixel pitch keeps 16 consecutive pixels'
    // fragment reads on distinct banks.  Plane-major otherwise.
    static constexpr bool PM = PM_;
    static constexpr int QS = PM ? 1 : HS, PS = PM ? 3 : 1;  // slots between planes / pixels
    static constexpr int WA = (PM ? 3 : 2) * HS;           // t0 weight slots [9][2][32]
    static constexpr int WB = WA + 9 * 2 * 32;             // t1 weight slots [9][2][64]
    static constexpr int ITEM = WB + 9 * 2 * 64;           // slots per item
    static constexpr int PPW = (ITEM + 64 * NW - 1) / (64 * NW);  // 1-KiB DMA pieces per wave per item
    static constexpr int BUF = PPW * NW * 1024;            // bytes per ring slot
    static constexpr int LDS = 2 * BUF + (32 + 64) * 4;    // + biases
    static constexpr int F0 = TH * W / 32;                 // t0 fragments per tile (24)
    static constexpr int H1 = TH / 2, W1 = W / 2;          // t1 rows / columns per tile
    static constexpr int F1 = H1 * W1 / 32;                // t1 fragments per tile (6)
    // waves 0-3 run t0 (6 fragments each), waves 4-7 t1 (one 32-cout group, 3 fragments each):
    // every SIMD hosts one wave of each role, 54 + 27 MFMAs per item (the former 6 + 2 split
    // put 90 on two SIMDs and 72 on the others)
    static constexpr int NF0 = 6, NF1 = 3;                 // fragments per t0 / t1 wave
    static constexpr int NFM = NF0 > NF1 ? NF0 : NF1;
    static constexpr int ST1 = 2 * NFM;                    // epilogue stores per wave (at most)
    static_assert(F0 == 4 * NF0 && F1 == 2 * NF1, "4 t0 waves x 6 fragments, 4 t1 waves (2 cout groups x 3)");
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(H % TH == 0 && C % 16 == 0, "tiling");
    static_assert(2 * PPW < 48 && ST1 < 48, "vmcnt range");
};

struct TrParams {
    const uint16_t* x;
    const uint16_t* wb;  // weight blob: w0 [32][3][3][256] at element w0_off, w1 [64][3][3][256] at w1_off
    int w0_off, w1_off;  // (one base pointer: per-piece source offsets stay 32-bit)
    const float* b0;
    const float* b1;
    uint16_t* y0;        // [N][64][48][32]
    uint16_t* y1;        // [N][32][24][64]
    const uint16_t* zero;
    int N, n_tiles;
    // the weight slots of every 16-channel chunk in LDS order (trans1_pack_weights): 1 KB
    // contiguous per weight DMA instruction instead of 64 scattered rows; nullptr: gather from wb
    const uint16_t* wimg;
    // x in chunk-planar layout [N][16][64][48][16] (the fused Bottleneck's planar output): a
    // 16-channel item's halo is then one contiguous run per row, and no item shares a cache line
    // with another (NHWC: 4 items per 128-B line, re-fetched from HBM when L2 evicts it between them)
    int planar;
};

template <bool PM>
__global__ __launch_bounds__(512, 1) void trans1_kernel(TrParams p) {
    using G = T1C<PM>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    constexpr int tiles_h = G::H / G::TH;
    const bool is_t1 = wave >= 4;
    const uint16_t* zl = p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8;

    // ---- per-lane DMA geometry of this wave's item pieces (fixed for the launch)
    // kind 1 halo: po = element offset from the tile's (crop, row -1, col 0) + chunk, hy = halo row;
    // kind 2: weight element offset in the blob (t0 or t1 slice; + chunk * 16 at issue time)
    // the t1 waves (4-7, half the MFMAs of a t0 wave) issue the item pieces of virtual waves
    // vw = wave & 3 and (wave & 3) + 4, the t0 waves none: after the item barrier the t0 wave of
    // each SIMD starts its MFMAs at once (tconv16.hip; 836 -> 811 us, profiles/r04_dma_split_ab.txt)
    const bool dma_wave = wave >= 4;
    int pk[2][G::PPW], po[2][G::PPW];
#pragma unroll
    for (int v = 0; v < 2; v++)
#pragma unroll
    for (int j = 0; j < G::PPW; j++) {
        const int s = (j * G::NW + (wave & 3) + 4 * v) * 64 + lane;
        int kind = 0, off = 0, hy = 0;
        if (s < G::WA) {
            const int q = PM ? s % 3 : s / G::HS, hs = PM ? s / 3 : s - q * G::HS;
            if (hs > 0 && q < 2) {
                const int t = hs - 1, yy = t / G::RS, xx = t - yy * G::RS;
                if (xx < G::W) {
                    kind = 1;
                    hy = yy;
                    off = (yy * G::W + xx) * (p.planar ? 16 : G::C) + q * 8;
                }
            }
        } else if (s < G::ITEM && p.wimg) {
            kind = 2;
            off = (s - G::WA) * 8;
        } else if (s < G::WB) {
            const int ws = s - G::WA, row = ws & 31, tq = ws >> 5;  // tq = tap * 2 + q
            kind = 2;
            off = p.w0_off + (row_cout(row) * 9 + (tq >> 1)) * G::C + (tq & 1) * 8;
        } else if (s < G::ITEM) {
            const int ws = s - G::WB, row = ws & 63, tq = ws >> 6;
            kind = 2;
            off = p.w1_off + (((row & ~31) | row_cout(row & 31)) * 9 + (tq >> 1)) * G::C + (tq & 1) * 8;
        }
        pk[v][j] = (kind << 8) | hy;
        po[v][j] = off;
    }
    auto issue = [&](int item, int buf) {
        const int tile = blockIdx.x + (item / G::NCH) * gridDim.x, chunk = item % G::NCH;
        const int n = tile / tiles_h, r0 = (tile - n * tiles_h) * G::TH;
        const uint16_t* xb = p.planar ? p.x + (((long)n * G::NCH + chunk) * G::H + r0 - 1) * G::W * 16
                                      : p.x + ((long)n * G::H + r0 - 1) * G::W * G::C + chunk * 16;
        uint8_t* dst = lds + buf * G::BUF;
        const uint16_t* wbase = p.wimg ? p.wimg + chunk * (G::ITEM - G::WA) * 8 : p.wb + chunk * 16;
        if (!dma_wave) return;
#pragma unroll
        for (int v = 0; v < 2; v++)
#pragma unroll
        for (int j = 0; j < G::PPW; j++) {
            const int vw = (wave & 3) + 4 * v;
            const int kind = pk[v][j] >> 8, hy = pk[v][j] & 255;
            const bool in = kind == 1 && (unsigned)(r0 - 1 + hy) < (unsigned)G::H;
            const uint16_t* src = kind == 2 ? wbase + po[v][j] : in ? xb + po[v][j] : zl;
            // pieces wholly past the item's slots are not issued (3 of 72)
            if (j < G::PPW - 1 || (j * G::NW + vw) * 64 < G::ITEM)
                glds16(src, dst + (j * G::NW + vw) * 1024);
        }
    };

    // ---- fragment geometry: t0 waves fragments f = wave * 4 + i, t1 waves f = i (cout group wave - 6)
    int bv[G::NFM], eo[G::NFM];
#pragma unroll
    for (int i = 0; i < G::NFM; i++) {
        if (!is_t1) {
            const int f = (i < G::NF0) ? wave * G::NF0 + i : 0;
            const int pp = frag_pixel<G::W, G::TH, 1>(f, r32);
            const int ty = pp / G::W, x = pp - ty * G::W;
            bv[i] = (h * G::QS + (ty * G::RS + x) * G::PS) * 16;  // tap (0,0) of (ty, x): pixel 1 + (ty-1+1)*RS + x-1
            eo[i] = ty * G::W + x;
        } else {
            const int fi = i < G::NF1 ? ((wave - 4) >> 1) * G::NF1 + i : 0;
            const int pp = fi * 32 + r32;                // t1: 8 rows x 24 columns, generic order
            const int ro = pp / G::W1, c = pp - ro * G::W1;
            bv[i] = (h * G::QS + (2 * ro * G::RS + 2 * c) * G::PS) * 16;  // y (2ro-1, 2c-1): pixel 1 + 2ro*RS + 2c - 1
            eo[i] = ro * G::W1 + c;
        }
    }
    const int mg1 = (wave - 4) & 1;
    const int av = is_t1 ? (G::WB + h * 64 + mg1 * 32 + r32) * 16 : (G::WA + h * 32 + r32) * 16;
    float* sbias = reinterpret_cast<float*>(lds + 2 * G::BUF);
    if (tid < 32) sbias[tid] = p.b0[tid];
    else if (tid < 96) sbias[tid] = p.b1[tid - 32];

    const int n_items = ((p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) * G::NCH;
    issue(0, 0);
    // one item loop per role (own accumulators, no register merges between the roles);
    // both loops run the same items and barriers
    auto loop = [&](auto nf_tag, auto t1_tag) {
        constexpr int NF = decltype(nf_tag)::value;
        constexpr bool S2C = decltype(t1_tag)::value;
        constexpr int AST = S2C ? 2 * 64 * 16 : 2 * 32 * 16;  // A bytes per tap
        f32x16 acc[NF];
        for (int k = 0; k < n_items; k++) {
            const int buf = k & 1, chunk = k % G::NCH;
            const bool first = chunk == 0, last = chunk == G::NCH - 1;
            // item k has landed (younger: only the previous tile's epilogue stores); the barrier
            // publishes every wave's pieces and retires all reads of the other ring slot
            if (k == 0)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else if (!first)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NF) : "memory");
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const int tile = blockIdx.x + (k / G::NCH) * gridDim.x;
            const int n = tile / tiles_h, r0 = (tile - n * tiles_h) * G::TH;
            if (first) {
                f32x16 b;
                const float4* bp = reinterpret_cast<const float4*>(sbias + (S2C ? 32 + mg1 * 32 : 0) + 16 * h);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float4 q = bp[j];
                    b[4 * j] = q.x;
                    b[4 * j + 1] = q.y;
                    b[4 * j + 2] = q.z;
                    b[4 * j + 3] = q.w;
                }
#pragma unroll
                for (int i = 0; i < NF; i++) acc[i] = b;
            }
            if (k + 1 < n_items) issue(k + 1, buf ^ 1);
            asm volatile("" ::: "memory");
            const int boff = buf * G::BUF;
            // 9 taps x 1 k-step (16 channels); fragments of tap t+1 read before tap t's MFMAs
            bf16x8 fa[2], fb[2][NF];
            auto load = [&](int tap, bf16x8& a, bf16x8 (&b)[NF]) {
                const int dy = tap / 3, dx = tap % 3;
                a = *reinterpret_cast<const bf16x8*>(lds + boff + av + tap * AST);
#pragma unroll
                for (int t = 0; t < NF; t++)
                    b[t] = *reinterpret_cast<const bf16x8*>(lds + boff + bv[t] + (dy * G::RS + dx) * G::PS * 16);
            };
            load(0, fa[0], fb[0]);
#pragma unroll
            for (int tap = 0; tap < 9; tap++) {
                const int cur = tap & 1;
                if (tap + 1 < 9) load(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < NF; t++)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur][t], acc[t], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (last) {
                uint16_t* base = S2C ? p.y1 + ((long)n * (G::H / 2) + r0 / 2) * G::W1 * 64 + mg1 * 32 + 16 * h
                                     : p.y0 + ((long)n * G::H + r0) * G::W * 32 + 16 * h;
#pragma unroll
                for (int t = 0; t < NF; t++) {
                    uint32_t o[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) o[e] = pack_bf16x2(relu1(acc[t][2 * e]), relu1(acc[t][2 * e + 1]));
                    uint16_t* yp = base + (long)eo[t] * (S2C ? 64 : 32);
                    *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
                    *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
                }
            }
        }
    };
    if (is_t1)
        loop(std::integral_constant<int, G::NF1>{}, std::true_type{});
    else
        loop(std::integral_constant<int, G::NF0>{}, std::false_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int g_tr_cus = 0;

}  // namespace

bool trans1_supported(int H, int W, int C, int cout0, int cout1) {
    const char* e = getenv("MVPOSE_NO_TRANSFUSE");  // diagnostics/tests: the two convs apart
    if (e && e[0] == '1') return false;
    return H == T1C<true>::H && W == T1C<true>::W && C == T1C<true>::C && cout0 == 32 && cout1 == 64;
}

// Weight image: per 16-channel chunk, t0's [tap][q][32 permuted couts] then t1's [tap][q][64]
// (the kernel's slots WA .. ITEM), 1,728 x 16 B; same element count as w0 + w1.
__global__ __launch_bounds__(256) void trans1_pack_kernel(const uint16_t* __restrict__ wb, int w0_off, int w1_off,
                                                          uint16_t* __restrict__ img) {
    constexpr int C = 256, NCH = C / 16, S0 = 9 * 2 * 32, SI = S0 + 9 * 2 * 64;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < NCH * SI; i += gridDim.x * 256) {
        const int chunk = i / SI, ws = i - chunk * SI;
        const uint16_t* src;
        if (ws < S0) {
            const int row = ws & 31, tq = ws >> 5;
            src = wb + w0_off + (row_cout(row) * 9 + (tq >> 1)) * C + (tq & 1) * 8;
        } else {
            const int w = ws - S0, row = w & 63, tq = w >> 6;
            src = wb + w1_off + (((row & ~31) | row_cout(row & 31)) * 9 + (tq >> 1)) * C + (tq & 1) * 8;
        }
        *reinterpret_cast<uint4*>(img + (long)i * 8) = *reinterpret_cast<const uint4*>(src + chunk * 16);
    }
}

void trans1_pack_weights(const uint16_t* wb, int64_t w0_off, int64_t w1_off, uint16_t* img, hipStream_t s) {
    static_assert(T1C<true>::ITEM - T1C<true>::WA == 9 * 2 * 96, "image item");
    hipLaunchKernelGGL(trans1_pack_kernel, dim3(108), dim3(256), 0, s, wb, (int)w0_off, (int)w1_off, img);
    MVP_HIP(hipGetLastError());
}

void launch_trans1(const uint16_t* x, const uint16_t* wb, int64_t w0_off, const float* b0, int64_t w1_off,
                   const float* b1, uint16_t* y0, uint16_t* y1, int N, hipStream_t s, const uint16_t* wimg,
                   bool planar) {
    MVP_REQUIRE(w0_off >= 0 && w1_off >= 0 && w0_off + 32 * 9 * 256 < (1LL << 31) && w1_off + 64 * 9 * 256 < (1LL << 31),
                "trans1: weight offsets exceed 32 bits");
    if (N == 0) return;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)trans1_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    T1C<true>::LDS));
        attr = true;
    }
    if (g_tr_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_tr_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long tiles = (long)N * (T1C<true>::H / T1C<true>::TH);
    MVP_REQUIRE(tiles * T1C<true>::NCH < (1L << 30), "trans1: too many tiles");
    TrParams p{x, wb, (int)w0_off, (int)w1_off, b0, b1, y0, y1, conv_zero_region(), N, (int)tiles, wimg, planar ? 1 : 0};
    const int grid = (int)std::min<long>(tiles, g_tr_cus);
    // pixel-major halo (+0.4 % frames/s over plane-major, round 2)
    hipLaunchKernelGGL(trans1_kernel<true>, dim3(grid), dim3(T1C<true>::NTH), T1C<true>::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
