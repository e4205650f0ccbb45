// Fused HRNet BasicBlock on the 64-channel 32x24 branch plane (gfx950), warp-specialised:
//   y = relu( conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x )
// for HRNet-W32's 32 BasicBlocks on branch 1 (64 ch @ 32x24).  Run as two tconv launches
// the block moves its 100 MB (1,024 crops) input twice and writes the intermediate once;
// fused, HBM sees the input (with a 4-row halo per 8 output rows) and the output only.
//
// One workgroup of 4 waves (one per SIMD) per CU, persistent over tiles of 8 output rows
// of one crop.  The waves specialise:
//   waves 0, 1  conv1 for output rows -1 .. 8 (10 rows: conv2's halo), cout group 0 / 1
//               -> the intermediate (bias, ReLU, bf16; rows outside the image = 0 = conv2's
//               zero padding) in LDS;
//   waves 2, 3  conv2 of the PREVIOUS tile from the other intermediate buffer, + b2 +
//               residual (global, issued before the DMA) + ReLU -> output, and the input
//               halo DMA of the NEXT tile into the idle ring slot.
// So each phase (one barrier) runs conv1 of tile k beside conv2 of tile k-1 on the other
// two SIMDs, and the halo of tile k+1 streams in under both.  Each wave keeps its conv's
// 32 couts x 576 K of weights in registers (144 VGPRs, loaded once per launch: no weight
// traffic in the loop and only B fragments are read from LDS, one ds_read_b128 per MFMA).
// LDS: input halo ring 2 x 42 KiB (channel pairs interleaved per pixel, as tblock32) +
// intermediate 2 x 31.4 KiB (plane-major, row pitch W+1 with a zero pad slot).
//
// Every accumulator sees tconv_kernel's MFMA sequence (bias start, K order (32-channel
// chunk, tap, 16-channel half)) and its epilogue, so the result is bit-identical to the two
// separate tconv launches (tests/test_backbone_gpu.py, tests/test_conv_planes_gpu.py).
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;  // 16-B slots of the shared zero region

struct B64 {
    static constexpr int H = 32, W = 24, TH = 8, RS = W + 1;
    static constexpr int TILES_H = H / TH;
    static constexpr int R1 = TH + 2;                         // conv1 rows (the intermediate)
    static constexpr int F1 = (R1 * W + 31) / 32;             // 8 fragments (the last 16 pixels pad)
    static constexpr int F2 = TH * W / 32;                    // 6 fragments
    static constexpr int HR = TH + 5;                         // input halo rows: 2 above, 2 below, 1 for the pad pixels
    static constexpr int HS = 1 + HR * RS;                    // input pixel slots (incl. the leading zero)
    static constexpr int HSM = 1 + R1 * RS;                   // intermediate slots per plane
    static constexpr int XSLOTS = 8 * HS;                     // 4 channel pairs x HS pixels x 2
    static constexpr int NDW = 2;                             // DMA-issuing waves
    static constexpr int XPPW = (XSLOTS + 64 * NDW - 1) / (64 * NDW);  // 1-KiB pieces per DMA wave
    static constexpr int XBYTES = XPPW * NDW * 1024;          // one input ring slot
    static constexpr int MBYTES = 8 * HSM * 16;               // one intermediate buffer
    static constexpr int MOFF = 2 * XBYTES;
    static constexpr int LDS = MOFF + 2 * MBYTES;
    static constexpr int KS = 36;                              // k-steps: 2 chunks x 9 taps x 2 halves
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(R1 * W > (F1 - 1) * 32 && F2 * 32 == TH * W, "fragments");
    static_assert((3 * 2 * HS + (2 * RS + 2) * 2) * 16 < 65536 && (7 * HSM + 2 * RS + 2) * 16 < 65536,
                  "ds_read offset range");
    static_assert(HR < 31 && 2 * F2 + XPPW < 64, "packed DMA geometry / vmcnt range");
};

struct TB64Params {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y;
    const uint16_t* zero;
    int N, n_tiles;
};

// Weights of one conv's cout group, in registers for the launch: A fragment of k-step
// s = (chunk c, tap, half ks) for lane (r32, h): cout 32cg + row_cout(r32), input channels
// 32c + 16ks + 8h .. +7 (tconv_kernel's K order).
__device__ __forceinline__ void load_weights(const uint16_t* __restrict__ w, int cg, int r32, int h,
                                             bf16x8 (&wa)[B64::KS]) {
    const int cout = 32 * cg + row_cout(r32);
#pragma unroll
    for (int s = 0; s < B64::KS; s++) {
        const int c = s / 18, tap = (s % 18) >> 1, ks = s & 1;
        wa[s] = *reinterpret_cast<const bf16x8*>(w + (cout * 9 + tap) * 64 + c * 32 + ks * 16 + 8 * h);
    }
}

// The accumulators start at the bias (couts 32cg + 16h .. +15), reloaded per tile (L2).
__device__ __forceinline__ f32x16 bias_acc(const float* __restrict__ b, int cg, int h) {
    const float* bp = b + 32 * cg + 16 * h;
    f32x16 a;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float4 b4 = *reinterpret_cast<const float4*>(bp + 4 * j);
        a[4 * j] = b4.x;
        a[4 * j + 1] = b4.y;
        a[4 * j + 2] = b4.z;
        a[4 * j + 3] = b4.w;
    }
    return a;
}

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// conv1 waves: tile k's 10 intermediate rows from input ring slot k & 1 into intermediate
// buffer k & 1, then the phase barrier.  n_items + 1 barriers, as the conv2 waves.
__device__ __forceinline__ void conv1_role(const TB64Params& p, uint8_t* lds, int cg, int lane, int n_items) {
    using G = B64;
    constexpr int W = G::W, H = G::H, TH = G::TH, RS = G::RS;
    const int h = lane >> 5, r32 = lane & 31;
    bf16x8 wa[G::KS];
    load_weights(p.w1, cg, r32, h, wa);
    // fragment t, lane r32: intermediate pixel pp = 32t + r32 of the 10 x 24 rows (pp >= 240:
    // padding pixels, computed on the spare halo row, never written)
    int bv1[G::F1], mw[G::F1];
#pragma unroll
    for (int t = 0; t < G::F1; t++) {
        const int pp = 32 * t + r32, r = pp / W, x = pp - (pp / W) * W;
        bv1[t] = ((r * RS + x) * 2 + h) * 16;                                  // input halo, tap (0, 0)
        mw[t] = G::MOFF + ((4 * cg + 2 * h) * G::HSM + 1 + r * RS + x) * 16;  // intermediate, plane 4cg + 2h
    }
    barrier();  // prologue: tile 0's halo and the zeroed intermediate
    for (int k = 0; k < n_items; k++) {
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / G::TILES_H, ho0 = (tile - n * G::TILES_H) * TH;
        f32x16 acc[G::F1];
        acc[0] = bias_acc(p.b1, cg, h);
#pragma unroll
        for (int t = 1; t < G::F1; t++) acc[t] = acc[0];
        const int xo = (k & 1) * G::XBYTES;
        bf16x8 fb[2][G::F1];
        auto load = [&](int s, bf16x8 (&b)[G::F1]) {
            const int c = s / 18, tap = (s % 18) >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < G::F1; t++)
                b[t] = *reinterpret_cast<const bf16x8*>(lds + xo + bv1[t] + ((c * 2 + ks) * 2 * G::HS) * 16 +
                                                        (dy * RS + dx) * 32);
        };
        load(0, fb[0]);
#pragma unroll
        for (int s = 0; s < G::KS; s++) {
            if (s + 1 < G::KS) load(s + 1, fb[(s + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < G::F1; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], fb[s & 1][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        const int mo = (k & 1) * G::MBYTES;
#pragma unroll
        for (int t = 0; t < G::F1; t++) {
            const int pp = 32 * t + r32;
            if (pp < G::R1 * W) {
                // rows outside the image are conv2's zero padding
                const bool live = (unsigned)(ho0 - 1 + pp / W) < (unsigned)H;
                uint32_t o[8];
#pragma unroll
                for (int e = 0; e < 8; e++)
                    o[e] = live ? pack_bf16x2(relu1(acc[t][2 * e]), relu1(acc[t][2 * e + 1])) : 0u;
                *reinterpret_cast<uint4*>(lds + mw[t] + mo) = uint4{o[0], o[1], o[2], o[3]};
                *reinterpret_cast<uint4*>(lds + mw[t] + mo + G::HSM * 16) = uint4{o[4], o[5], o[6], o[7]};
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
    }
    barrier();  // the conv2 waves' last phase
}

// Input halo of tile k into ring slot buf, by the two conv2 waves (dw = 0, 1): ring slot
// 16-B slot s = pair pp, pixel pix, plane e -> channels 16pp + 8e of halo pixel pix (0 = the
// leading zero; row hy = image row ho0 - 2 + hy; column hx = W is the zero pad).
__device__ __forceinline__ void issue_halo(const TB64Params& p, uint8_t* lds, int dw, int lane, const uint16_t* zl,
                                           int k, int buf) {
    using G = B64;
    constexpr int W = G::W, H = G::H, TH = G::TH, RS = G::RS;
    const int tile = blockIdx.x + k * gridDim.x;
    const int n = tile / G::TILES_H, ho0 = (tile - n * G::TILES_H) * TH;
    const uint16_t* xb = p.x + ((long)n * H + ho0) * W * 64;
#pragma unroll
    for (int j = 0; j < G::XPPW; j++) {
        const int s = (j * G::NDW + dw) * 64 + lane;
        const int pp = s / (2 * G::HS), rem = s - pp * (2 * G::HS), pix = rem >> 1, e = rem & 1;
        const int t = pix - 1, hy = t / RS, hx = t - hy * RS;
        const bool in = s < G::XSLOTS && pix > 0 && hx < W && (unsigned)(ho0 + hy - 2) < (unsigned)H;
        glds16(in ? xb + ((hy - 2) * W + hx) * 64 + pp * 16 + e * 8 : zl,
               lds + buf * G::XBYTES + (j * G::NDW + dw) * 1024);
    }
}

// conv2 waves: in phase k, the residual of tile k-1 (global), the halo DMA of tile k+1, conv2
// of tile k-1 from intermediate buffer (k-1) & 1 + bias + residual + ReLU -> y.
__device__ __forceinline__ void conv2_role(const TB64Params& p, uint8_t* lds, int cg, int lane, int n_items,
                                           const uint16_t* zl) {
    using G = B64;
    constexpr int W = G::W, H = G::H, TH = G::TH, RS = G::RS;
    const int h = lane >> 5, r32 = lane & 31, dw = cg;
    bf16x8 wa[G::KS];
    load_weights(p.w2, cg, r32, h, wa);
    int bv2[G::F2];
#pragma unroll
    for (int t = 0; t < G::F2; t++) {
        const int pp = 32 * t + r32, r = pp / W, x = pp - (pp / W) * W;
        bv2[t] = G::MOFF + (h * G::HSM + r * RS + x) * 16;  // intermediate, tap (0, 0), plane h
    }
    issue_halo(p, lds, dw, lane, zl, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();  // prologue
    for (int k = 0; k <= n_items; k++) {
        const bool conv = k >= 1, dma = k + 1 < n_items;
        if (!conv) {
            if (dma) issue_halo(p, lds, dw, lane, zl, k + 1, (k + 1) & 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier();
            continue;
        }
        const int kp = k - 1;
        const int tile = blockIdx.x + kp * gridDim.x;
        const int n = tile / G::TILES_H, ho0 = (tile - n * G::TILES_H) * TH;
        const long pix0 = ((long)n * H + ho0) * W;
        f32x16 acc[G::F2];
        acc[0] = bias_acc(p.b2, cg, h);
        // the residual, issued before the DMA so the epilogue never waits for the halo
        uint4 rv[G::F2][2];
#pragma unroll
        for (int t = 0; t < G::F2; t++) {
            const uint16_t* rs = p.x + (pix0 + 32 * t + r32) * 64 + 32 * cg + 16 * h;
            rv[t][0] = *reinterpret_cast<const uint4*>(rs);
            rv[t][1] = *reinterpret_cast<const uint4*>(rs + 8);
        }
#pragma unroll
        for (int t = 1; t < G::F2; t++) acc[t] = acc[0];
        asm volatile("" ::: "memory");
        if (dma) issue_halo(p, lds, dw, lane, zl, k + 1, (k + 1) & 1);
        asm volatile("" ::: "memory");
        const int mo = (kp & 1) * G::MBYTES;
        bf16x8 fb[2][G::F2];
        auto load = [&](int s, bf16x8 (&b)[G::F2]) {
            const int c = s / 18, tap = (s % 18) >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < G::F2; t++)
                b[t] = *reinterpret_cast<const bf16x8*>(lds + mo + bv2[t] +
                                                        ((c * 4 + ks * 2) * G::HSM + dy * RS + dx) * 16);
        };
        load(0, fb[0]);
#pragma unroll
        for (int s = 0; s < G::KS; s++) {
            if (s + 1 < G::KS) load(s + 1, fb[(s + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < G::F2; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], fb[s & 1][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        // the residual loads are older than the DMA pieces
        if (dma)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::XPPW) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < G::F2; t++) {
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint4 rr = rv[t][e >> 2];
                const uint32_t u = (e & 3) == 0 ? rr.x : (e & 3) == 1 ? rr.y : (e & 3) == 2 ? rr.z : rr.w;
                o[e] = pack_bf16x2(relu1(acc[t][2 * e] + lo_bf16(u)), relu1(acc[t][2 * e + 1] + hi_bf16(u)));
            }
            uint16_t* yp = p.y + (pix0 + 32 * t + r32) * 64 + 32 * cg + 16 * h;
            *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
        }
        // the next tile's halo has landed (only this tile's stores may still be in flight)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::F2) : "memory");
        barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256, 1) void tblock64_kernel(TB64Params p) {
    using G = B64;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    const int n_items = (p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    // the intermediate's pad and leading slots stay zero for the launch
    for (int i = tid; i < 2 * G::MBYTES / 16; i += 256)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (wave < 2)
        conv1_role(p, lds, wave, lane, n_items);
    else
        conv2_role(p, lds, wave - 2, lane, n_items, p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8);
}

int g_tb64_cus = 0;

}  // namespace

bool tblock64_supported(int H, int W) {
    const char* e = getenv("MVPOSE_NO_TBLOCK64");  // A/B and tests: two tconv launches instead
    return !(e && e[0] == '1') && H == B64::H && W == B64::W;
}

void launch_tblock64(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                     uint16_t* y, int N, int H, int W, hipStream_t s) {
    using G = B64;
    MVP_REQUIRE(H == G::H && W == G::W, "tblock64: unsupported plane %dx%d", H, W);
    if (N == 0) return;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)tblock64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (g_tb64_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_tb64_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long tiles = (long)N * G::TILES_H;
    MVP_REQUIRE(tiles < (1L << 30), "tblock64: too many tiles");
    TB64Params p{x, w1, b1, w2, b2, y, conv_zero_region(), N, (int)tiles};
    const int grid = (int)std::min<long>(tiles, g_tb64_cus);
    hipLaunchKernelGGL(tblock64_kernel, dim3(grid), dim3(256), G::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
