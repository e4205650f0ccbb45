// Streaming fused HRNet Bottleneck on layer1's 256-channel 64x48 plane (gfx950):
//   y = relu( conv1x1(relu(conv3x3(relu(conv1x1(x, w1) + b1), w2) + b2), w3) + b3 + x )
// (x, y: 256 ch; the two intermediates: 64 ch).  Layer1's blocks 2-4 ran as a 3x3 tconv
// launch plus a Bottleneck join (conv3 + the next block's conv1, conv1x1_pair_kernel): per
// block 0.4 GB of 64-ch intermediates were written and read back beside the 1.6 GB 256-ch
// tensor's read and write (4.8 GB per 1,024 crops).  Here the block reads x once and writes y
// once (3.2 GB); the intermediates live in LDS.
//
// * One workgroup per CU (8 waves) walks WHOLE crops top to bottom, two output rows per
//   step.  x rows arrive by LDS-DMA into a 5-row ring (24 KiB per row) one step ahead of
//   use; a row stays resident from conv1 (which reads it) to conv3 (whose residual it is),
//   and conv3's output overwrites its residual in place, so the ring row is also the
//   output's staging buffer: the next step stores it with whole-1-KiB coalesced writes and
//   refills the slot with the DMA of a later row.
// * Warp-specialised, weights in VGPRs for the launch.  Waves 0-3 (C13): conv1 (wave j:
//   couts 16j..16j+15, 16x16x32 MFMAs over the row's 3 pixel tiles) into a 4-row ring of
//   the 64-ch intermediate, then conv3 (wave j: couts 64j..64j+63) + b3 + residual + ReLU.
//   Waves 4-7 (C2): conv2 on 32x32x16 MFMAs (wave 4 + gr: 32-cout group gr, fragments 0 and
//   2 of the step's 96 pixels; waves 6-7: fragment 1), and the step's row stores and DMAs.
//   Phases (one barrier each): P1 conv1 | stores + DMA, P2 conv2, P3 conv3.
// * x ring rows are pixel-major (512 B per pixel) with the 16-B chunk index XOR-swizzled by
//   the pixel (bn_swz): a DMA / store instruction moves 2 whole pixels (1 KiB contiguous in
//   HBM), and both conv1's B-fragment reads and conv3's residual reads are conflict-free.
//
// Numerics (bit-identical to the unfused graph): conv1 sums K in the pair kernel's order
// (perm = 1: its second GEMM's permuted chunks, the graph's Bottleneck-join path) or the
// 1x1 kernel's (perm = 0), from 0, + b1, ReLU, bf16; conv2 = tconv_kernel's sequence
// (accumulators start at b2; chunk, tap, 16-channel half), ReLU, bf16; conv3 = the pair
// kernel's first GEMM (2 chunks from 0) + b3 + residual, ReLU, bf16.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// LEAD: layer1's first block — x is the stem's 64-ch output and conv3 is cat-fused with the
// downsample (K = [conv2's 64 | x's 64], no residual; graph cat_fuse).  x rows are then 6 KiB
// and stay in an 8-row ring until conv3 has read them.
template <bool LEAD>
struct BNT {
    static constexpr int H = 64, W = 48, M = 64, CO = 256;
    static constexpr int C = LEAD ? 64 : 256;       // x channels
    static constexpr int XROW = W * C * 2;          // one x row: 24 KiB (6 KiB)
    static constexpr int NX = LEAD ? 8 : 5;         // x ring rows
    static constexpr int PIECES = XROW / 1024;      // 1-KiB DMA pieces per row (2 or 8 pixels each)
    static constexpr int RS = W + 1;                // intermediate row pitch (slots; slot 48 is zero)
    static constexpr int TR = 4;                    // intermediate ring rows
    static constexpr int TPL = (1 + TR * RS) * 16;  // one 8-channel plane of the ring (leading zero slot)
    static constexpr int TOFF = NX * XROW;
    static constexpr int T2PL = 2 * W * 16;         // one 8-channel plane of conv2's output (2 rows)
    static constexpr int T2OFF = TOFF + 8 * TPL;
    static constexpr int BOFF = T2OFF + 8 * T2PL;   // biases (f32): conv2's 64 | conv1's 64 | conv3's 256
    static constexpr int LDS = BOFF + (64 + 64 + 256) * 4;
    static constexpr int STEPS = H / 2;             // 2 output rows per step
    static constexpr int KS = 36;                   // conv2 k-steps: 2 chunks x 9 taps x 2 halves
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(7 * TPL + 32 < 65536 && 2 * 8192 + 256 < 65536, "ds_read offset range");
};

constexpr int wait_vm(int n) { return ((n >> 4) << 14) | 0x0F70 | (n & 15); }
constexpr int kWaitLgkm0 = 0xC07F;

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// x-ring swizzle: chunk c16 of pixel p sits at slot p * 32 + ((c16 & 16) | ((c16 & 15) ^ bn_swz(p))).
// ds_read_b128 serves lanes {0-3, 12-15, 20-27} (and the complementary set) together: conv1's
// fragment lanes (pixel px, 16-channel group g) and conv3's residual lanes then hit 16
// distinct bank groups for every chunk (mfma_tile.h, lane_rank).
__device__ __forceinline__ int bn_swz(int p) {
    const int x = p & 15;
    return x < 4 ? x : x < 12 ? x + 4 : x - 8;
}
// LEAD (8 chunks per pixel): chunk c16 at slot p * 8 + (c16 ^ ((p >> 1) & 7)), conflict-free for
// the same fragment lanes (checked by brute force over the lane groups)
template <bool LEAD>
__device__ __forceinline__ int xoff(int p, int c16) {
    if constexpr (LEAD)
        return p * 128 + ((c16 ^ (p >> 1)) & 7) * 16;
    else
        return p * 512 + ((c16 & 16) | ((c16 & 15) ^ bn_swz(p))) * 16;
}
// The row DMA as raw instructions: through the builtin, the compiler treats the LDS-DMA as an
// LDS store of unknown extent and waits for it (vmcnt(0)) before the next LDS read, which put
// the whole DMA latency in front of conv2.  The ring protocol orders it instead: a slot is
// refilled only after the barrier that retired its readers, and published by the explicit
// vmcnt wait before the barrier that precedes its next reader.  lds_off: byte offset in the
// dynamic LDS (the kernel has no static LDS), wave-uniform; lane i writes lds_off + 16 i.
__device__ __forceinline__ void glds16_ring(const void* src, uint32_t lds_off) {
    uint32_t saved;  // m0 is the compiler's: restored after the issue (the DMA reads it at issue)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(src), "s"(lds_off)
        : "memory");
}

// x ring slot of row r of crop-local index cl (rows of a workgroup's crops in stream order)
template <bool LEAD>
__device__ __forceinline__ int xslot(int cl, int r) {
    using BN = BNT<LEAD>;
    return (cl * BN::H + r) % BN::NX;
}

#ifdef BNECK_STAMPS  // timing harness (tools/bneck_stamps.py): workgroup 0's phase times, in y
#define BN_STAMP(s, b)                                                                                     \
    do {                                                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                       \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (s) < 128)                                       \
            reinterpret_cast<unsigned long long*>(p.y)[((threadIdx.x >> 6) * 128 + (s)) * 8 + (b)] = t_; \
    } while (0)
#else
#define BN_STAMP(s, b) \
    do {               \
    } while (0)
#endif

struct BNParams {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    const uint16_t* w3;
    const float* b3;
    uint16_t* y;
    int N, perm, planar;
};

// ------------------------------------------------------------------ C2 waves
// Piece n = jw + 4m of a row holds pixels 2n, 2n + 1; lane -> (pixel 2n + (lane >> 5), chunk
// c16): the element offset within the row is 512 m + lane_off(m & 1) (pixel & 15 depends on m's
// parity only).
__device__ __forceinline__ int piece_lane_off(int jw, int lane, int odd) {
    const int px = 2 * jw + (lane >> 5), cs = lane & 31;  // pixel of piece jw (m = 0)
    return px * 256 + ((cs & 16) | ((cs & 15) ^ bn_swz(px + 8 * odd))) * 8;
}

// x rows conv1 reads in step s (all but the first of a crop: 2, the crop's last: 1)
__device__ __forceinline__ int step_rows(int s) {
    const int k = s % 32;
    return k == 0 ? 3 : k == 31 ? 1 : 2;
}
// DMA instructions wave jw issues per row: 24 pieces on 4 waves, or (LEAD) 6 pieces: 2, 2, 1, 1
template <bool LEAD>
__device__ __forceinline__ int wave_pieces(int jw) {
    return LEAD ? (jw < 2 ? 2 : 1) : BNT<false>::PIECES / 4;
}
// s_waitcnt vmcnt(n) for a runtime n <= 18
__device__ __forceinline__ void wait_vm_dyn(int n) {
    switch (n) {
#define BN_W(k) \
    case k: __builtin_amdgcn_s_waitcnt(wait_vm(k)); break;
        BN_W(1) BN_W(2) BN_W(3) BN_W(4) BN_W(5) BN_W(6) BN_W(7) BN_W(8) BN_W(9) BN_W(10) BN_W(11) BN_W(12)
        BN_W(13) BN_W(14) BN_W(15) BN_W(16) BN_W(17) BN_W(18)
#undef BN_W
        default: __builtin_amdgcn_s_waitcnt(wait_vm(0)); break;
    }
}

// Row traffic of step s (x rows conv1 reads in it): rows 0-2 of the crop at its first step,
// rows 2k+1, 2k+2 (< 64) after.  Wave jw moves pieces jw, jw + 4, ... of each row.
template <bool LEAD>
__device__ __forceinline__ void dma_step(const BNParams& p, int crop0, int s, int jw, int lane) {
    using BN = BNT<LEAD>;
    const int cl = s / BN::STEPS, k = s - cl * BN::STEPS;
    const int r0 = k == 0 ? 0 : 2 * k + 1, r1 = k == 0 ? 3 : min(2 * k + 3, BN::H);
    if constexpr (LEAD) {
        // piece n = jw, jw + 4 (< 6): pixels 8n .. 8n + 7, lane -> pixel 8n + (lane >> 3), chunk slot lane & 7
        for (int r = r0; r < r1; r++) {
            const uint16_t* src = p.x + ((long)(crop0 + cl) * BN::H + r) * BN::W * BN::C;
            const uint32_t dst = xslot<LEAD>(cl, r) * BN::XROW;
            for (int n = jw; n < BN::PIECES; n += 4) {
                const int px = 8 * n + (lane >> 3), c16 = ((lane & 7) ^ (px >> 1)) & 7;
                glds16_ring(src + px * BN::C + c16 * 8, __builtin_amdgcn_readfirstlane(dst + n * 1024));
            }
        }
    } else {
        const int lo0 = piece_lane_off(jw, lane, 0), lo1 = piece_lane_off(jw, lane, 1);
        for (int r = r0; r < r1; r++) {
            const uint16_t* src = p.x + ((long)(crop0 + cl) * BN::H + r) * BN::W * BN::C;
            const uint32_t dst = xslot<LEAD>(cl, r) * BN::XROW + jw * 1024;
#pragma unroll
            for (int m = 0; m < BN::PIECES / 4; m++)
                glds16_ring(src + 2048 * m + ((m & 1) ? lo1 : lo0), __builtin_amdgcn_readfirstlane(dst + m * 4096));
        }
    }
}

#ifndef BNECK_PF2
#define BNECK_PF2 3
#endif

template <bool LEAD>
__device__ __forceinline__ void c2_role(const BNParams& p, uint8_t* lds, int jw, int lane, int crop0, int n_steps) {
    using BN = BNT<LEAD>;
    constexpr int kPF = BNECK_PF2;
    const int h = lane >> 5, r32 = lane & 31, gr = jw & 1, fr = jw >> 1;
    // A fragments, k-step s = chunk * 18 + tap * 2 + half: W2[cout][tap][32 chunk + 16 half + 8h .. +7]
    bf16x8 wa[BN::KS];
    {
        const int cout = gr * 32 + row_cout(r32);
#pragma unroll
        for (int s = 0; s < BN::KS; s++) {
            const int c = s / 18, tap = (s % 18) >> 1, ks = s & 1;
            wa[s] = *reinterpret_cast<const bf16x8*>(p.w2 + (cout * 9 + tap) * BN::M + c * 32 + ks * 16 + 8 * h);
        }
    }
    // fragments of the step's 96 pixels (2 rows, row-major): waves 4-5 take 0 and 2, waves 6-7 take 1
    int fpp[2];
#pragma unroll
    for (int t = 0; t < 2; t++) fpp[t] = frag_pixel<BN::W, 2, 1>(fr == 0 ? 2 * t : 1, r32);

    // conv2 of step k's rows: NF fragments (waves 4-5: 0 and 2; waves 6-7: 1)
    auto conv2 = [&](auto nf_tag, int k) {
        constexpr int NF = decltype(nf_tag)::value;
        int bv[NF][3];
#pragma unroll
        for (int t = 0; t < NF; t++) {
            const int rho = fpp[t] / BN::W, x = fpp[t] - rho * BN::W;
#pragma unroll
            for (int dy = 0; dy < 3; dy++)  // + dx * 16: column x + dx - 1
                bv[t][dy] = BN::TOFF + h * BN::TPL + (((2 * k + rho + dy) & 3) * BN::RS + x) * 16;
        }
        // accumulators start at the lane's 16 biases (couts 32gr + 16h ..), from LDS
        f32x16 acc[NF];
        {
            const float4* bq = reinterpret_cast<const float4*>(lds + BN::BOFF + (gr * 32 + 16 * h) * 4);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 b4 = bq[q];
                acc[0][4 * q] = b4.x;
                acc[0][4 * q + 1] = b4.y;
                acc[0][4 * q + 2] = b4.z;
                acc[0][4 * q + 3] = b4.w;
            }
#pragma unroll
            for (int t = 1; t < NF; t++) acc[t] = acc[0];
        }
        bf16x8 fb[kPF + 1][NF];
        auto load = [&](auto Ss) {
            constexpr int st = Ss, c = st / 18, tap = (st % 18) >> 1, ks = st & 1;
            constexpr int dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < NF; t++)
                fb[st % (kPF + 1)][t] =
                    *reinterpret_cast<const bf16x8*>(lds + bv[t][dy] + ((4 * c + 2 * ks) * BN::TPL + dx * 16));
        };
        static_for<0, kPF>(load);
        static_for<0, BN::KS>([&](auto Ss) {
            constexpr int st = Ss;
            if constexpr (st + kPF < BN::KS) load(std::integral_constant<int, st + kPF>{});
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < NF; t++)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[st], fb[st % (kPF + 1)][t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        });
        // ReLU, bf16 -> conv2's output planes (lane: couts 32gr + 16h .. +15 of its pixel)
#pragma unroll
        for (int t = 0; t < NF; t++) {
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) o[e] = pack_bf16x2(relu1(acc[t][2 * e]), relu1(acc[t][2 * e + 1]));
            uint8_t* d = lds + BN::T2OFF + (4 * gr + 2 * h) * BN::T2PL + fpp[t] * 16;
            *reinterpret_cast<uint4*>(d) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(d + BN::T2PL) = uint4{o[4], o[5], o[6], o[7]};
        }
    };

    dma_step<LEAD>(p, crop0, 0, jw, lane);
    if (n_steps > 1) dma_step<LEAD>(p, crop0, 1, jw, lane);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    barrier();  // prologue: steps 0 and 1's rows, the zeroed intermediate ring
    for (int s = 0; s < n_steps; s++) {
        BN_STAMP(s, 0);
        // ---- P1: the conv1 waves read step s's rows
        barrier();
        BN_STAMP(s, 2);
        // ---- P2: conv2 of rows 2k, 2k+1 from intermediate rows 2k-1 .. 2k+2 (the conv1/conv3
        // waves issue the row DMAs meanwhile)
        if (fr == 0)
            conv2(std::integral_constant<int, 2>{}, s % BN::STEPS);
        else
            conv2(std::integral_constant<int, 1>{}, s % BN::STEPS);
        __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
        BN_STAMP(s, 3);
        barrier();
        BN_STAMP(s, 4);
        // ---- P3: the conv1/conv3 waves run conv3
        BN_STAMP(s, 5);
        barrier();
    }
}

// ------------------------------------------------------------------ C13 waves
// conv3's output lanes: wave j, lane group g owns two runs of 8 couts, chunks cap(g, 0..1) —
// the x chunks conv1's lane (px, g) reads as its K chunks 2j and 2j+1 — so the residual of a
// row is read once, beside conv1's fragments, while the row is in the ring, and kept in VGPRs
// until conv3 of that row; the x ring then holds rows only until conv1 has read them.
__device__ __forceinline__ int cap_chunk(int perm, int j, int g, int e) {
    return perm ? 16 * (j >> 1) + 4 * g + 2 * (j & 1) + e : 4 * (2 * j + e) + g;
}

struct Resid {
    uint4 v[3][2];  // [pixel tile][run]
};

template <bool LEAD>
__device__ __forceinline__ void c13_role(const BNParams& p, uint8_t* lds, int j, int lane, int crop0, int n_steps) {
    using BN = BNT<LEAD>;
    constexpr int KC1 = BN::C / 32;  // conv1 K chunks: 8 (2 for LEAD: the 1x1 kernel's natural order)
    const int px = lane & 15, g = lane >> 4;
    // conv1: wave j computes couts 32 (j & 1) .. + 31 (two 16-cout tiles: A row px of tile c ->
    // cout 32 (j & 1) + 16c + px) of one of the step's two rows (j >> 1), so each x fragment is
    // read by two waves, not four; the lane's x-ring chunk offsets per K chunk jc
    const int cb = 32 * (j & 1), half = j >> 1;
    bf16x8 w1f[2][KC1];
    int xo[LEAD ? 2 : 4];  // chunk jc at xo[jc & 3] + 256 (jc >> 2) in either K order (LEAD: xo[jc])
#pragma unroll
    for (int jc = 0; jc < KC1; jc++) {
        const int c16 = (p.perm && !LEAD) ? 16 * (jc >> 2) + 4 * g + (jc & 3) : 4 * jc + g;
#pragma unroll
        for (int c = 0; c < 2; c++)
            w1f[c][jc] = *reinterpret_cast<const bf16x8*>(p.w1 + (cb + 16 * c + px) * BN::C + c16 * 8);
        if (jc < (LEAD ? 2 : 4)) xo[jc] = xoff<LEAD>(px, c16);
    }
    // conv3 A, tile ct, row r (D lane group r >> 2): LEAD -> cout 64j + 16 (r >> 2) + 4ct + (r & 3)
    // over K = 128 (4 chunks: conv2's output, then x); else -> cout 8 cap(r >> 2, ct >> 1) +
    // 4 (ct & 1) + (r & 3) over K = 64
    constexpr int KC3 = LEAD ? 4 : 2;
    bf16x8 w3f[4][KC3];
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
        for (int ch = 0; ch < KC3; ch++) {
            const int cout = LEAD ? 64 * j + 16 * (px >> 2) + 4 * ct + (px & 3)
                                  : 8 * cap_chunk(p.perm, j, px >> 2, ct >> 1) + 4 * (ct & 1) + (px & 3);
            w3f[ct][ch] = *reinterpret_cast<const bf16x8*>(p.w3 + cout * (32 * KC3) + ch * 32 + 8 * g);
        }
    int cap[2], ro[2];  // the lane's two 8-cout output runs (chunks) and their x-ring offsets
#pragma unroll
    for (int e = 0; e < 2; e++) {
        cap[e] = LEAD ? 8 * j + 2 * g + e : cap_chunk(p.perm, j, g, e);
        ro[e] = LEAD ? 0 : xoff<LEAD>(px, cap[e]);
    }
    const float* b1s = reinterpret_cast<const float*>(lds + BN::BOFF) + 64;
    const float* b3s = b1s + 64;
    __builtin_amdgcn_s_waitcnt(wait_vm(0));

    // intermediate row r (-1 .. 64) of the current crop: ring row (r + 1) & 3
    // (this wave's 4 planes of it)
    auto zero_row = [&](int r) {
        const int pos = (r + 1) & 3;
        for (int i = lane; i < 4 * BN::W; i += 64) {
            const int q = 4 * (j & 1) + i / BN::W, x = i % BN::W;
            *reinterpret_cast<uint4*>(lds + BN::TOFF + q * BN::TPL + (1 + pos * BN::RS + x) * 16) =
                uint4{0u, 0u, 0u, 0u};
        }
    };
    // the residual of x row r for conv3 (this wave's couts), while the row is in the ring
    auto resid_row = [&](int cl, int r, Resid& res) {
        if constexpr (!LEAD) {
            const uint8_t* xb = lds + xslot<LEAD>(cl, r) * BN::XROW;
#pragma unroll
            for (int t = 0; t < 3; t++)
#pragma unroll
                for (int e = 0; e < 2; e++) res.v[t][e] = *reinterpret_cast<const uint4*>(xb + ro[e] + t * 8192);
        }
    };
    // pixel tile t of an x row in the ring: + t * XTILE
    constexpr int XTILE = 16 * BN::C * 2;
    auto conv1_row = [&](int cl, int r) {
        const uint8_t* xb = lds + xslot<LEAD>(cl, r) * BN::XROW;
        f32x4 acc[2][3];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int t = 0; t < 3; t++) acc[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        // chunk jc+1's fragments are read while chunk jc's 6 MFMAs run
        bf16x8 b[2][3];
        auto load = [&](auto Jc) {
            constexpr int jc = Jc;
            const int off = LEAD ? xo[jc & 1] : xo[jc & 3] + (jc >> 2) * 256;
#pragma unroll
            for (int t = 0; t < 3; t++) b[jc & 1][t] = *reinterpret_cast<const bf16x8*>(xb + off + t * XTILE);
        };
        load(std::integral_constant<int, 0>{});
        static_for<0, KC1>([&](auto Jc) {
            constexpr int jc = Jc;
            if constexpr (jc + 1 < KC1) load(std::integral_constant<int, jc + 1>{});
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int c = 0; c < 2; c++)
#pragma unroll
                for (int t = 0; t < 3; t++)
                    acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[c][jc], b[jc & 1][t], acc[c][t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        });
        const int pos = (r + 1) & 3;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const float4 bb = *reinterpret_cast<const float4*>(b1s + cb + 16 * c + 4 * g);
            const float b1v[4] = {bb.x, bb.y, bb.z, bb.w};
            uint8_t* d = lds + BN::TOFF + (4 * (j & 1) + 2 * c + (g >> 1)) * BN::TPL + (1 + pos * BN::RS + px) * 16 +
                         (g & 1) * 8;
#pragma unroll
            for (int t = 0; t < 3; t++) {
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = fmaxf(acc[c][t][i] + b1v[i], 0.f);
                *reinterpret_cast<uint2*>(d + t * 256) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
            }
        }
    };
    // conv3 of output row r (rho = its row in the step) + b3 + residual + ReLU -> y
    auto conv3_row = [&](int cl, int k, int rho, const Resid& res) {
        uint16_t* yrow = p.y + ((long)(crop0 + cl) * BN::H + 2 * k + rho) * BN::W * BN::CO;
        float b3v[16];
#pragma unroll
        for (int e = 0; e < 2; e++)
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const float4 bb = *reinterpret_cast<const float4*>(b3s + 8 * cap[e] + 4 * q);
                b3v[8 * e + 4 * q] = bb.x;
                b3v[8 * e + 4 * q + 1] = bb.y;
                b3v[8 * e + 4 * q + 2] = bb.z;
                b3v[8 * e + 4 * q + 3] = bb.w;
            }
        const uint8_t* tb = lds + BN::T2OFF + g * BN::T2PL + (rho * BN::W + px) * 16;
        // LEAD: K chunks 2-3 are the block input's (x row 2k + rho, still in the ring)
        const uint8_t* xb = lds + xslot<LEAD>(cl, 2 * k + rho) * BN::XROW;
        bf16x8 bq[2][KC3];  // [tile parity][chunk]: the next tile's fragments read during this one
        auto load = [&](int tc, bf16x8(&dst)[KC3]) {
#pragma unroll
            for (int ch = 0; ch < 2; ch++) dst[ch] = *reinterpret_cast<const bf16x8*>(tb + 4 * ch * BN::T2PL + tc * 256);
            if constexpr (LEAD) {
#pragma unroll
                for (int ch = 2; ch < KC3; ch++)
                    dst[ch] = *reinterpret_cast<const bf16x8*>(xb + xo[ch - 2] + tc * XTILE);
            }
        };
        load(0, bq[0]);
#pragma unroll
        for (int tc = 0; tc < 3; tc++) {
            if (tc + 1 < 3) load(tc + 1, bq[(tc + 1) & 1]);
            const bf16x8(&bch)[KC3] = bq[tc & 1];
            f32x4 acc[4];
#pragma unroll
            for (int ct = 0; ct < 4; ct++) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ch = 0; ch < KC3; ch++)
#pragma unroll
                for (int ct = 0; ct < 4; ct++)
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3f[ct][ch], bch[ch], acc[ct], 0, 0, 0);
            uint32_t o[8];
            if constexpr (LEAD) {  // cat-fused downsample: no residual
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int ct = q >> 1, i = 2 * (q & 1);
                    o[q] = pack_bf16x2(fmaxf(acc[ct][i] + b3v[2 * q], 0.f), fmaxf(acc[ct][i + 1] + b3v[2 * q + 1], 0.f));
                }
            } else {
                const uint4 r0 = res.v[tc][0], r1 = res.v[tc][1];
                const uint32_t rw[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int ct = q >> 1, i = 2 * (q & 1);
                    float v0 = acc[ct][i] + b3v[2 * q], v1 = acc[ct][i + 1] + b3v[2 * q + 1];
                    v0 += lo_bf16(rw[q]);
                    v1 += hi_bf16(rw[q]);
                    o[q] = pack_bf16x2(fmaxf(v0, 0.f), fmaxf(v1, 0.f));
                }
            }
#ifdef BNECK_STAMPS
            if (blockIdx.x == 0) continue;
#endif
            uint16_t* yq[2];
            if (!LEAD && p.planar) {  // [crop][16-ch chunk][row][col][16]
                const int row = 2 * k + rho, col = tc * 16 + px;
#pragma unroll
                for (int e = 0; e < 2; e++)
                    yq[e] = p.y + ((((long)(crop0 + cl) * 16 + (cap[e] >> 1)) * BN::H + row) * BN::W + col) * 16 +
                            (cap[e] & 1) * 8;
            } else {
                uint16_t* yp = yrow + (tc * 16 + px) * BN::CO;
#pragma unroll
                for (int e = 0; e < 2; e++) yq[e] = yp + cap[e] * 8;
            }
            *reinterpret_cast<uint4*>(yq[0]) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(yq[1]) = uint4{o[4], o[5], o[6], o[7]};
        }
    };

    Resid r_lo, r_hi, r_next;  // residuals of rows 2k, 2k+1, 2k+2
    barrier();  // prologue
    for (int s = 0; s < n_steps; s++) {
        const int cl = s / BN::STEPS, k = s - cl * BN::STEPS;
        BN_STAMP(s, 0);
        // ---- P1: conv1 of intermediate rows 2k+1, 2k+2 (first step: -1 (zero), 0, 1, 2)
        if (k == 0) {
            resid_row(cl, 0, r_lo);
            resid_row(cl, 1, r_hi);
            resid_row(cl, 2, r_next);
            if (half == 0) {
                conv1_row(cl, 0);
                conv1_row(cl, 2);
            } else {
                zero_row(-1);
                conv1_row(cl, 1);
            }
        } else {
            if constexpr (!LEAD) r_lo = r_next;
            resid_row(cl, 2 * k + 1, r_hi);
            if (2 * k + 2 < BN::H) resid_row(cl, 2 * k + 2, r_next);
            if (half == 0)
                conv1_row(cl, 2 * k + 1);
            else if (2 * k + 2 < BN::H)
                conv1_row(cl, 2 * k + 2);
            else
                zero_row(BN::H);
        }
        __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
        BN_STAMP(s, 1);
        barrier();
        BN_STAMP(s, 2);
        // ---- P2: conv2 (the C2 waves).  This wave issues its share of the DMA of step s+2's
        // rows into the slots step s's conv1 has just released (and the one step s-1 released;
        // LEAD: slots conv3 has released):
        // the issue (~100 cycles per 1-KiB instruction) stays off the conv2 waves' critical path.
        // (Issued by the conv2 waves during conv3 instead, it leaves conv2's LDS reads alone but
        // has a step less lead: 714 -> 836 us per block.)
#ifndef BNECK_DIAG_NO_DMA  // timing harness only (stale rows, wrong results)
        if (s + 2 < n_steps) dma_step<LEAD>(p, crop0, s + 2, j, lane);
#endif
        barrier();
        BN_STAMP(s, 4);
        // ---- P3: step s+1's rows (issued a step ago) land before the barrier that ends this
        // step; step s+2's stay in flight.  Waited before conv3's stores, so that only DMAs are
        // younger than the counted ones.
        wait_vm_dyn(s + 2 < n_steps ? step_rows(s + 2) * wave_pieces<LEAD>(j) : 0);
        // ---- P3: conv3 of rows 2k, 2k+1
        conv3_row(cl, k, 0, r_lo);
        conv3_row(cl, k, 1, r_hi);
        __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
        BN_STAMP(s, 5);
        barrier();
    }
}

template <bool LEAD>
__global__ __launch_bounds__(512, 1) void bneck_kernel(BNParams p) {
    using BN = BNT<LEAD>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nb = gridDim.x, b = blockIdx.x;
    const int crop0 = (int)(((long)p.N * b) / nb), crop1 = (int)(((long)p.N * (b + 1)) / nb);
    const int n_steps = (crop1 - crop0) * BN::STEPS;
    if (n_steps == 0) return;  // whole workgroup: uniform
    // the intermediate ring (its leading and pad slots stay zero)
    for (int i = tid; i < 8 * BN::TPL / 16; i += 512)
        *reinterpret_cast<uint4*>(lds + BN::TOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    for (int i = tid; i < 64 + 64 + 256; i += 512)
        reinterpret_cast<float*>(lds + BN::BOFF)[i] = i < 64 ? p.b2[i] : i < 128 ? p.b1[i - 64] : p.b3[i - 128];
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    if (wave < 4)
        c13_role<LEAD>(p, lds, wave, lane, crop0, n_steps);
    else
        c2_role<LEAD>(p, lds, wave - 4, lane, crop0, n_steps);
}

int g_bn_cus = 0;

}  // namespace

bool bneck_supported(int H, int W, int C, int M) {
    const char* e = getenv("MVPOSE_NO_BNECK");  // tests / A/B: the tconv + Bottleneck-join path
    if (e && e[0] == '1') return false;
    using BN = BNT<false>;
    return H == BN::H && W == BN::W && (C == BNT<false>::C || C == BNT<true>::C) && M == BN::M;
}

template <bool LEAD>
void launch_bneck_t(const BNParams& p, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)bneck_kernel<LEAD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    BNT<LEAD>::LDS));
        attr = true;
    }
    const int grid = std::min(p.N, g_bn_cus);
    hipLaunchKernelGGL(bneck_kernel<LEAD>, dim3(grid), dim3(512), BNT<LEAD>::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

void launch_bneck(const BneckLaunch& c, hipStream_t s) {
    MVP_REQUIRE(c.H == BNT<false>::H && c.W == BNT<false>::W, "bneck: plane %dx%d", c.H, c.W);
    MVP_REQUIRE(c.N >= 0 && c.N < (1 << 24), "bneck: %d crops", c.N);
    if (c.N == 0) return;
    if (g_bn_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_bn_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    MVP_REQUIRE(!(c.lead && c.planar), "bneck: planar output is for the 256-ch blocks");
    BNParams p{c.x, c.w1, c.b1, c.w2, c.b2, c.w3, c.b3, c.y, c.N, c.perm ? 1 : 0, c.planar ? 1 : 0};
    if (c.lead)
        launch_bneck_t<true>(p, s);
    else
        launch_bneck_t<false>(p, s);
}

}  // namespace mvp
