// Fused HRNet BasicBlock on the 64-channel 32x24 branch plane (gfx950), warp-specialised:
//   y = relu( conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x )
// for HRNet-W32's 32 BasicBlocks on branch 1 (64 ch @ 32x24).  Run as two tconv launches
// the block moves its 100 MB (1,024 crops) input twice and writes the intermediate once;
// fused, HBM sees the input (with a 4-row halo per 8 output rows) and the output only.
//
// One workgroup of 4 waves (one per SIMD) per CU, persistent over a contiguous range of
// crops, each crop's 4 tiles of 8 output rows top to bottom (round 4: tiles 1-3 of a crop copy
// their first two intermediate rows from the previous tile instead of recomputing them, 8 -> 6
// conv1 fragments; 120 -> 114.5 us per block, profiles/r04_tblock64_rowreuse_ab.txt).  The
// waves specialise:
//   waves 0, 1  conv1 for output rows -1 .. 8 (10 rows: conv2's halo), half of the
//               fragments each -> the intermediate (bias, ReLU, bf16; rows outside the
//               image = 0 = conv2's zero padding) in LDS;
//   waves 2, 3  conv2 of the PREVIOUS tile from the other intermediate buffer, half of the
//               fragments each, + b2 + residual (read from the input ring) + ReLU ->
//               output, and the input halo DMA of the NEXT tile into the idle ring slot.
// So each phase (one barrier) runs conv1 of tile k beside conv2 of tile k-1 on the other
// two SIMDs, and the halo of tile k+1 streams in under both.  Each wave keeps its conv's
// 64 couts x 576 K of weights in registers (288 of the 512 a lone wave per SIMD has, AGPRs
// included; loaded once per launch) and computes BOTH 32-cout groups of its fragments, so
// every B fragment read from LDS feeds two MFMAs (round 5; with one cout group per wave
// each MFMA had its own ds_read_b128 and LDS reads bound the kernel: 129 -> 123 us per
// block, profiles/r05_tb64_2cg_ab.txt).
//
// LDS images (input halo ring 2 x 40 KiB, intermediate 2 x 32.5 KiB) are plane-major
// (8 planes of 8 channels, 16-B slots) with a row pitch of 26 slots (zero pad | 24 pixels |
// zero pad).  A fragment's 32 pixels are an 8-row x 4-column block whose even rows go to
// one ds_read_b128 lane group of the half-wave ({0-3,12-15,20-27}) and odd rows to the
// other: with the pitch = 10 (mod 16) every group reads 16 distinct bank quads for every
// tap, so the B-operand reads are conflict-free (the first layout — channel pairs
// interleaved per pixel, raster fragments across the pad slots — measured 2.6-way,
// SQ_LDS_BANK_CONFLICT 56 % of the LDS cycles).  conv1's rows 8-9 use 2 x 16 blocks.
//
// Every accumulator sees tconv_kernel's MFMA sequence (bias start, K order (32-channel
// chunk, tap, 16-channel half)) and its epilogue, so the result is bit-identical to the two
// separate tconv launches (tests/test_conv_planes_gpu.py, tests/test_backbone_gpu.py).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "conv.h"
#include "mfma_tile.h"
#include "mvp_common.h"

namespace mvp {
namespace {

using namespace mfma_tile;

constexpr int kZeroSlots = 4096;  // 16-B slots of the shared zero region

struct B64 {
    static constexpr int H = 32, W = 24, TH = 8, RS = W + 2;
    static constexpr int TILES_H = H / TH;
    static constexpr int R1 = TH + 2;            // conv1 rows (the intermediate)
    static constexpr int F1 = 8;                 // 6 blocks of 8x4 (rows 0-7) + 2 of 2x16 (rows 8-9)
    static constexpr int F2 = 6;                 // 6 blocks of 8x4
    static constexpr int HR = TH + 4;            // input halo rows: 2 above, 2 below
    static constexpr int HSP = 320;              // input slots per plane (HR * RS = 312 used; 64-slot DMA blocks)
    static constexpr int HSM = R1 * RS;          // intermediate slots per plane
    static constexpr int NB = (HSP + 63) / 64;   // 64-slot DMA blocks per plane
    static constexpr int NPIECE = 8 * NB;        // 1-KiB DMA pieces per tile
    static constexpr int NDW = 2;                // DMA-issuing waves
    static constexpr int XPPW = NPIECE / NDW;    // pieces per DMA wave
    static constexpr int XBYTES = 8 * HSP * 16;  // one ring slot
    static constexpr int MBYTES = 8 * HSM * 16;  // one intermediate buffer
    static constexpr int MOFF = 2 * XBYTES;
    static constexpr int BOFF = MOFF + 2 * MBYTES;  // b1 | b2 (f32)
    static constexpr int LDS = BOFF + 2 * 64 * 4;
    static constexpr int KS = 36;                // k-steps: 2 chunks x 9 taps x 2 halves
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(RS % 16 == 10, "conflict-free 8x4 blocks need a row pitch of 10 (mod 16)");
    static_assert(HSP >= HR * RS && HSP % 64 == 0 && HSP % 16 == 0, "plane stride: whole DMA blocks, bank-neutral");
    static_assert(NPIECE % NDW == 0 && 2 * F2 + XPPW < 64 && XPPW == 4 * NB, "DMA split / vmcnt range");
    static_assert(F1 == 8 && F2 == 6, "fragment split: conv1 4 + 4 (3 + 3 shifted), conv2 3 + 3 per wave");
    static_assert((6 * HSP + 2 * RS + 2) * 16 < 65536 && (6 * HSM + 2 * RS + 2) * 16 < 65536, "ds_read offset range");
};

// Intermediate / output pixel (row r, column x) of fragment t for lane r32; pad = a
// duplicate lane of conv1's last fragment (reads a real lane's address, never written).
__device__ __forceinline__ void frag_pixel64(int t, int r32, int& r, int& x, bool& pad) {
    pad = false;
    if (t < 6) {
        r = blk_row(r32);
        x = 4 * t + blk_col(r32);
    } else {
        r = 8 + lane_grp(r32);
        const int pos = lane_pos(r32);
        x = t == 6 ? pos : 16 + (pos & 7);
        pad = t == 7 && pos >= 8;
    }
}

// s_waitcnt through the builtin, so the compiler's own wait insertion sees it (an asm
// s_waitcnt is opaque: the weight loads issued before the tile loop then looked pending on
// every iteration and put a vmcnt(0) in front of the first MFMA).  gfx9 encoding: vmcnt in
// bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8.
constexpr int wait_vm(int n) { return ((n >> 4) << 14) | 0x0F70 | (n & 15); }
constexpr int kWaitLgkm0 = 0xC07F;
constexpr int kWaitAll = 0x0070;

struct TB64Params {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y;
    const uint16_t* zero;
    int N, n_tiles;
#ifdef TB64_STAMPS
    unsigned long long* stamps;  // [block][wave][4] s_memtime segment sums (tools/tb64_stamps.hip)
#endif
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

// The accumulators start at the bias (couts 32cg + 16h .. +15), read per tile from the LDS
// copy.  Inline asm with its own lgkmcnt wait: as a plain LDS load the compiler puts a
// vmcnt(0) in front of it (the previous phase's halo DMA is an LDS write it cannot see
// completed), which in the conv2 waves also waited for the residual loads just issued.
__device__ __forceinline__ f32x16 bias_acc(const uint8_t* lds, int conv, int cg, int h) {
    const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(lds) + B64::BOFF + (64 * conv + 32 * cg + 16 * h) * 4;
    float4 q0, q1, q2, q3;
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %4 offset:16\n\t"
        "ds_read_b128 %2, %4 offset:32\n\t"
        "ds_read_b128 %3, %4 offset:48\n\t"
        "s_waitcnt lgkmcnt(0)"  // (this asm's own wait: the compiler does not track these reads)
        : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)  // early clobber: not the address register
        : "v"(a)
        : "memory");
    f32x16 r;
    const float4 q[4] = {q0, q1, q2, q3};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        r[4 * j] = q[j].x;
        r[4 * j + 1] = q[j].y;
        r[4 * j + 2] = q[j].z;
        r[4 * j + 3] = q[j].w;
    }
    return r;
}

#ifdef TB64_STAMPS
// Per-wave segment sums of s_memtime (tools/tb64_stamps.hip): stamp i closes segment i - 1 of
// the phase (stamp 0 the role's last one); wave-uniform scalars, written once at the role's end
// (per-phase stamps stored to memory needed VGPRs the two-group kernel does not have).
#define TB64_STAMP_DECL(ns)                                     \
    constexpr int tb_ns_ = (ns);                                \
    unsigned long long tb_sum_[4] = {0, 0, 0, 0}, tb_last_ = 0; \
    bool tb_on_ = false
#define TB64_STAMP(k, i)                                                  \
    do {                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
        if ((i) > 0)                                                      \
            tb_sum_[(i) > 0 ? (i) - 1 : 0] += t_ - tb_last_;              \
        else if (tb_on_)                                                  \
            tb_sum_[tb_ns_ - 1] += t_ - tb_last_;                         \
        tb_on_ = true;                                                    \
        tb_last_ = t_;                                                    \
    } while (0)
#define TB64_STAMP_FLUSH()                                                                        \
    do {                                                                                          \
        if ((threadIdx.x & 63) == 0)                                                              \
            for (int i_ = 0; i_ < 4; i_++)                                                        \
                p.stamps[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + i_] = tb_sum_[i_];  \
    } while (0)
#else
#define TB64_STAMP_DECL(ns) \
    do {                    \
    } while (0)
#define TB64_STAMP(k, i) \
    do {                 \
    } while (0)
#define TB64_STAMP_FLUSH() \
    do {                   \
    } while (0)
#endif

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Compile-time loop: f(std::integral_constant<int, i>) for i in [B, E) — the step index is a
// constant expression inside f (waitcnt immediates, buffer and fragment selection).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Both roles run their K loop as 72 steps: the first 36 accumulate the fragments of half A,
// the last 36 those of half B (weights in registers, so the split costs no extra reads),
// with the B operand prefetched PF = 2 steps ahead across the halves.  Half A's epilogue
// (bias is already in the accumulator; ReLU, bf16, store) runs in the MFMA shadow of half
// B's steps; only half B's epilogue is exposed.
#ifndef TB64_PF
#define TB64_PF 2
#endif
constexpr int kPF = TB64_PF;

// Tile k of this workgroup: crop and strip.  ST (strided, small batches): tile
// blockIdx.x + k * gridDim.x, conv1 computing every row; else a contiguous crop range.
// A template parameter so the crop-range kernel's code is unchanged by the strided mode.
template <bool ST>
__device__ __forceinline__ void tile_of64(int crop0, int k, int& n, int& s) {
    using G = B64;
    if (ST) {
        const int t = (int)blockIdx.x + k * (int)gridDim.x;
        n = t / G::TILES_H;
        s = t - n * G::TILES_H;
    } else {
        n = crop0 + k / G::TILES_H;
        s = k % G::TILES_H;
    }
}

// conv1 waves (w = 0, 1): tile k's intermediate rows from input ring slot k & 1 into
// intermediate buffer k & 1, then the phase barrier.  n_items + 2 barriers, as the conv2
// waves.  A workgroup walks its crops' 4 tiles top to bottom, so tile k's intermediate rows
// 0-1 (output rows ho0 - 1, ho0) are tile k-1's rows 8-9: for s > 0 they are copied from the
// other buffer and only rows 2-9 are computed (6 fragments of 8x4 blocks); the first tile of a
// crop computes all 10 rows (8 fragments, rows 0-7 as blocks, 8-9 as 2x16).  With crop ranges
// (NCG = 2) wave w computes BOTH cout groups of half the fragments (4w .. 4w+3 of the full
// set, 3w .. 3w+2 of the shifted one): each B fragment read from LDS feeds two MFMAs (round 5:
// with one cout group per wave, one ds_read_b128 per MFMA made LDS the bound -- a timing probe
// reading half the fragments ran 134 -> 96 us per block, profiles/r05_tb64_2cg_ab.txt).  The
// strided mode (one or two tiles per workgroup) keeps one cout group per wave (NCG = 1: cout
// group w, every fragment): there the twice-as-large weight load of the 2-group form is not
// amortised (40 crops: 20.8 -> 24.1 us per block).  Same MFMA sequence per accumulator in
// every form: bit-identical.  Half A's epilogues at steps 40 + 7j.
template <bool ST>
__device__ __forceinline__ void conv1_role(const TB64Params& p, uint8_t* lds, int w, int lane, int n_items,
                                           int crop0) {
    using G = B64;
    constexpr int H = G::H, TH = G::TH, RS = G::RS, CGB = 4 * G::HSM * 16;  // cout group 1: planes 4-7
    constexpr int NCG = ST ? 1 : 2, FF = G::F1 / NCG, FS = 6 / NCG, PF = kPF;
    const int h = lane >> 5, r32 = lane & 31;
    TB64_STAMP_DECL(3);
    auto cg_of = [&](int ci) { return NCG == 2 ? ci : w; };
    bf16x8 wa[NCG][G::KS];
#pragma unroll
    for (int ci = 0; ci < NCG; ci++) load_weights(p.w1, cg_of(ci), r32, h, wa[ci]);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    // fragment t, lane r32: intermediate pixel (r, x); its input tap (0, 0) is halo pixel
    // (r, x - 1) = slot r * RS + x, and it lands in intermediate slot r * RS + x + 1 (cout
    // group 0's planes; group 1's are CGB bytes on).  Full set (first tile of a crop):
    // frag_pixel64; shifted set (s > 0): 8x4 blocks at rows 2-9.
    int bvf[FF], mwf[FF], rf[FF], bvs[FS], mws[FS], rs3[FS];
#pragma unroll
    for (int t = 0; t < FF; t++) {
        int r, x;
        bool pad;
        frag_pixel64((NCG == 2 ? 4 * w : 0) + t, r32, r, x, pad);
        bvf[t] = (h * G::HSP + r * RS + x) * 16;
        mwf[t] = pad ? -1 : G::MOFF + (2 * h * G::HSM + r * RS + x + 1) * 16;
        rf[t] = r;
    }
    {  // fragment t of the shifted set is fragment 0's block moved 4 columns per step
        const int r = 2 + blk_row(r32), x = (NCG == 2 ? 12 * w : 0) + blk_col(r32);
        const int bv0 = (h * G::HSP + r * RS + x) * 16, mw0 = G::MOFF + (2 * h * G::HSM + r * RS + x + 1) * 16;
#pragma unroll
        for (int t = 0; t < FS; t++) {
            bvs[t] = bv0 + 64 * t;
            mws[t] = mw0 + 64 * t;
            rs3[t] = r;
        }
    }
    // one tile: NA fragments in half A, NB in half B, NCG cout groups each
    auto tile_body = [&](auto na_tag, auto nb_tag, const int* bv1, const int* mw, const int* rr, int k, int ho0) {
        constexpr int NA = decltype(na_tag)::value, NB = decltype(nb_tag)::value, NM = NA > NB ? NA : NB;
        f32x16 accA[NA][NCG], accB[NB][NCG];
#pragma unroll
        for (int ci = 0; ci < NCG; ci++) {
            accA[0][ci] = bias_acc(lds, 0, cg_of(ci), h);
#pragma unroll
            for (int t = 0; t < NB; t++) accB[t][ci] = accA[0][ci];
#pragma unroll
            for (int t = 1; t < NA; t++) accA[t][ci] = accA[0][ci];
        }
        const int xo = (k & 1) * G::XBYTES, mo = (k & 1) * G::MBYTES;
        bf16x8 fb[PF + 1][NM];
        auto load = [&](auto Gs) {  // B operands of step g (half g / 36, k-step g % 36)
            constexpr int g = Gs, s = g % 36, t0 = g < 36 ? 0 : NA, nt = g < 36 ? NA : NB;
            constexpr int c = s / 18, tap = (s % 18) >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < nt; t++)
                fb[g % (PF + 1)][t] = *reinterpret_cast<const bf16x8*>(
                    lds + xo + bv1[t0 + t] + ((4 * c + 2 * ks) * G::HSP + dy * RS + dx) * 16);
        };
        auto epilogue = [&](int t, int ci, const f32x16& a) {
            if (mw[t] < 0) return;
            // rows outside the image are conv2's zero padding
            const bool live = (unsigned)(ho0 - 1 + rr[t]) < (unsigned)H;
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) o[e] = live ? pack_bf16x2(relu1(a[2 * e]), relu1(a[2 * e + 1])) : 0u;
            uint8_t* d = lds + mw[t] + mo + cg_of(ci) * CGB;
            *reinterpret_cast<uint4*>(d) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(d + G::HSM * 16) = uint4{o[4], o[5], o[6], o[7]};
        };
        static_for<0, PF>(load);
        static_for<0, 72>([&](auto Gs) {
            constexpr int g = Gs, s = g % 36;
            if constexpr (g + PF < 72) load(std::integral_constant<int, g + PF>{});
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g < 36) {
#pragma unroll
                for (int t = 0; t < NA; t++)
#pragma unroll
                    for (int ci = 0; ci < NCG; ci++)
                        accA[t][ci] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ci][s], fb[g % (PF + 1)][t], accA[t][ci], 0, 0, 0);
            } else {
#pragma unroll
                for (int t = 0; t < NB; t++)
#pragma unroll
                    for (int ci = 0; ci < NCG; ci++)
                        accB[t][ci] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ci][s], fb[g % (PF + 1)][t], accB[t][ci], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g >= 40 && (g - 40) % 7 == 0 && (g - 40) / 7 < NCG * NA) {
                constexpr int j = (g - 40) / 7;
                epilogue(j / NCG, j % NCG, accA[j / NCG][j % NCG]);
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        TB64_STAMP(k, 1);
#pragma unroll
        for (int t = 0; t < NB; t++)
#pragma unroll
            for (int ci = 0; ci < NCG; ci++) epilogue(NA + t, ci, accB[t][ci]);
    };
    barrier();  // prologue: tile 0's halo and the zeroed intermediate
    for (int k = 0; k < n_items; k++) {
        TB64_STAMP(k, 0);
        int n_, s;
        tile_of64<ST>(crop0, k, n_, s);
        const int ho0 = s * TH;
        if (s == 0 || ST) {  // strided tiles: no previous tile of the crop in the other buffer
            tile_body(std::integral_constant<int, FF / 2>{}, std::integral_constant<int, FF / 2>{}, bvf, mwf, rf, k, ho0);
        } else {
            // rows 0-1 = the previous tile's rows 8-9 (planes 4w .. 4w+3, pads included)
            const int mo = (k & 1) * G::MBYTES, mp = ((k - 1) & 1) * G::MBYTES;
            for (int i = lane; i < 4 * 2 * RS; i += 64) {
                const int q = 4 * w + i / (2 * RS), rem = i % (2 * RS), r = rem / RS, xs = rem - r * RS;
                const int so = G::MOFF + (q * G::HSM + r * RS + xs) * 16;
                *reinterpret_cast<uint4*>(lds + so + mo) =
                    *reinterpret_cast<const uint4*>(lds + so + mp + 8 * RS * 16);
            }
            tile_body(std::integral_constant<int, NCG == 2 ? 2 : 3>{}, std::integral_constant<int, NCG == 2 ? 1 : 3>{}, bvs,
                      mws, rs3, k, ho0);
        }
        __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
        TB64_STAMP(k, 2);
        barrier();
    }
    barrier();  // the conv2 waves' last phase
    TB64_STAMP_FLUSH();
}

// Input halo of tile k into ring slot buf, by the two conv2 waves (dw = 0, 1).  Piece
// (block b, plane q) fills ring slots q * HSP + 64 b + lane with plane q of halo pixel
// p = 64 b + lane: row hy = p / RS (image row ho0 - 2 + hy), column p % RS - 1 (0 and RS - 1
// are the zero pads; p >= HR * RS is unused).  Wave dw issues planes dw, dw + 2, dw + 4,
// dw + 6 of every block, block-major (piece j = 4 b + q / 2), so a block's lane addresses
// are computed once and its 8 planes (the same 128-B pixel lines) are fetched together.
// valid = false (no tile k): zeros, so every phase issues the same VMEM ops.
struct HaloSrc {
    const uint16_t* xb;
    int ho0, buf;
    bool valid;
};
template <bool ST>
__device__ __forceinline__ HaloSrc halo_src(const TB64Params& p, int crop0, int k, int buf, bool valid) {
    using G = B64;
    int n, s;
    tile_of64<ST>(crop0, k, n, s);
    const int ho0 = s * G::TH;
    return HaloSrc{p.x + ((long)n * G::H + ho0) * G::W * 64, ho0, buf, valid};
}
__device__ __forceinline__ const uint16_t* halo_block(const HaloSrc& hs, int lane, const uint16_t* zl, int b) {
    using G = B64;
    const int px = 64 * b + lane, hy = px / G::RS, hx = px - hy * G::RS - 1;
    const bool in = hs.valid && px < G::HR * G::RS && (unsigned)hx < (unsigned)G::W &&
                    (unsigned)(hs.ho0 + hy - 2) < (unsigned)G::H;
    return in ? hs.xb + ((hy - 2) * G::W + hx) * 64 : zl;  // + 8 q per plane (zl: 64 KiB of zeros)
}
// The piece as raw instructions: through the builtin the compiler treats the LDS-DMA as an LDS
// store of unknown extent and drained every LDS read (lgkmcnt(0)) at each k-step it shared
// with a piece, exposing the B-fragment prefetch.  The ring protocol orders it instead: the
// slot a phase fills is read by no one in that phase (the residual reads of the slot precede
// the first piece, with their lgkmcnt wait), and the vmcnt wait before the phase barrier
// publishes it.  m0 is the compiler's: saved and restored around the issue.
__device__ __forceinline__ void glds16_raw(const void* src, uint32_t lds_off) {
    uint32_t saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(src), "s"(lds_off)
        : "memory");
}
__device__ __forceinline__ void halo_piece(const HaloSrc& hs, const uint16_t* blk, uint8_t* lds, int dw, int j) {
    using G = B64;
    const int b = j / 4, q = 2 * (j % 4) + dw;
    const uint32_t off = (uint32_t)reinterpret_cast<uintptr_t>(lds) + hs.buf * G::XBYTES + (q * G::HSP + 64 * b) * 16;
    glds16_raw(blk + q * 8, __builtin_amdgcn_readfirstlane(off));
}
__device__ __forceinline__ void issue_halo(const HaloSrc& hs, uint8_t* lds, int dw, int lane, const uint16_t* zl) {
    const uint16_t* blk = nullptr;
#pragma unroll
    for (int j = 0; j < B64::XPPW; j++) {
        if (j % 4 == 0) blk = halo_block(hs, lane, zl, j / 4);
        halo_piece(hs, blk, lds, dw, j);
    }
}

// conv2 schedule over the 72 steps: DMA piece j at step 1 + 2j (all before the first
// output store, so the phase-end vmcnt wait counts only stores); half A's epilogues (2
// fragments x 2 cout groups; strided mode: 3 x 1) at steps 40 + 7j.
constexpr int kDmaStep0 = 1, kDmaStride = 2;
static_assert(kDmaStep0 + kDmaStride * (B64::XPPW - 1) < 40, "DMA pieces precede the stores");

// conv2 waves (w = 0, 1): in phase k, the halo DMA of tile k+1 (planes w, w + 2, ...) and
// conv2 of tile k-1 from intermediate buffer (k-1) & 1 + bias + residual (from the input ring)
// + ReLU -> y: both cout groups of fragments 3w .. 3w+2 (half A: 2 fragments, half B: 1), or in
// the strided mode (NCG = 1) cout group w of all 6 fragments (3 + 3).
template <bool ST>
__device__ __forceinline__ void conv2_role(const TB64Params& p, uint8_t* lds, int w, int lane, int n_items,
                                           const uint16_t* zl, int crop0) {
    using G = B64;
    constexpr int W = G::W, H = G::H, TH = G::TH, RS = G::RS, PF = kPF;
    constexpr int NCG = ST ? 1 : 2, NF = G::F2 / NCG, NA = NCG == 2 ? 2 : 3, NB = NF - NA, NM = NA > NB ? NA : NB;
    const int h = lane >> 5, r32 = lane & 31, dw = w, f0 = NCG == 2 ? 3 * w : 0;
    TB64_STAMP_DECL(4);
    auto cg_of = [&](int ci) { return NCG == 2 ? ci : w; };
    bf16x8 wa[NCG][G::KS];
#pragma unroll
    for (int ci = 0; ci < NCG; ci++) load_weights(p.w2, cg_of(ci), r32, h, wa[ci]);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    // fragment t, lane r32: output pixel (r, x) = (blk_row, 4 (f0 + t) + blk_col); its tap
    // (0, 0) is intermediate pixel (r, x - 1) = slot r * RS + x
    int bv2[NF];
    const int er = blk_row(r32), ex = blk_col(r32);
#pragma unroll
    for (int t = 0; t < NF; t++) bv2[t] = G::MOFF + (h * G::HSM + er * RS + 4 * f0 + ex) * 16 + 64 * t;
    issue_halo(halo_src<ST>(p, crop0, 0, 0, true), lds, dw, lane, zl);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    barrier();  // prologue
    issue_halo(halo_src<ST>(p, crop0, 1, 1, n_items > 1), lds, dw, lane, zl);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    barrier();  // phase 0: conv1 of tile 0 only
    for (int k = 1; k <= n_items; k++) {
        TB64_STAMP(k, 0);
        const int kp = k - 1;
        int n, sp;
        tile_of64<ST>(crop0, kp, n, sp);
        const int ho0 = sp * TH;
        const long pix0 = ((long)n * H + ho0) * W;
        f32x16 accA[NA][NCG], accB[NB][NCG];
#pragma unroll
        for (int ci = 0; ci < NCG; ci++) accA[0][ci] = bias_acc(lds, 1, cg_of(ci), h);
        // the residual = tile k-1's input, still in ring slot (k-1) & 1 (halo rows 2-9): read
        // before this phase's DMA pieces start overwriting that slot with tile k+1
        uint4 rv[NF][NCG][2];
        {
            const uint8_t* rb = lds + (kp & 1) * G::XBYTES + (2 * h * G::HSP + (er + 2) * RS + ex + 1) * 16;
#pragma unroll
            for (int t = 0; t < NF; t++)
#pragma unroll
                for (int ci = 0; ci < NCG; ci++) {
                    const uint8_t* q = rb + (4 * cg_of(ci) * G::HSP + 4 * (f0 + t)) * 16;
                    rv[t][ci][0] = *reinterpret_cast<const uint4*>(q);
                    rv[t][ci][1] = *reinterpret_cast<const uint4*>(q + G::HSP * 16);
                }
        }
#pragma unroll
        for (int ci = 0; ci < NCG; ci++) {
#pragma unroll
            for (int t = 0; t < NB; t++) accB[t][ci] = accA[0][ci];
#pragma unroll
            for (int t = 1; t < NA; t++) accA[t][ci] = accA[0][ci];
        }
        __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
        __builtin_amdgcn_sched_barrier(0);
        const HaloSrc hn = halo_src<ST>(p, crop0, k + 1, (k + 1) & 1, k + 1 < n_items);
        const uint16_t* blk = nullptr;
        const int mo = (kp & 1) * G::MBYTES;
        bf16x8 fb[PF + 1][NM];
        auto load = [&](auto Gs) {
            constexpr int g = Gs, s = g % 36, t0 = g < 36 ? 0 : NA, nt = g < 36 ? NA : NB;
            constexpr int c = s / 18, tap = (s % 18) >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < nt; t++)
                fb[g % (PF + 1)][t] = *reinterpret_cast<const bf16x8*>(
                    lds + mo + bv2[t0 + t] + ((4 * c + 2 * ks) * G::HSM + dy * RS + dx) * 16);
        };
        auto epilogue = [&](int t, int ci, const f32x16& a) {
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint4 rr = rv[t][ci][e >> 2];
                const uint32_t u = (e & 3) == 0 ? rr.x : (e & 3) == 1 ? rr.y : (e & 3) == 2 ? rr.z : rr.w;
                o[e] = pack_bf16x2(relu1(a[2 * e] + lo_bf16(u)), relu1(a[2 * e + 1] + hi_bf16(u)));
            }
            uint16_t* yp = p.y + (pix0 + er * W + 4 * (f0 + t) + ex) * 64 + 32 * cg_of(ci) + 16 * h;
            *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
        };
        static_for<0, PF>(load);
        static_for<0, 72>([&](auto Gs) {
            constexpr int g = Gs, s = g % 36;
            if constexpr (g + PF < 72) load(std::integral_constant<int, g + PF>{});
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g < 36) {
#pragma unroll
                for (int t = 0; t < NA; t++)
#pragma unroll
                    for (int ci = 0; ci < NCG; ci++)
                        accA[t][ci] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ci][s], fb[g % (PF + 1)][t], accA[t][ci], 0, 0, 0);
            } else {
#pragma unroll
                for (int t = 0; t < NB; t++)
#pragma unroll
                    for (int ci = 0; ci < NCG; ci++)
                        accB[t][ci] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ci][s], fb[g % (PF + 1)][t], accB[t][ci], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g >= kDmaStep0 && (g - kDmaStep0) % kDmaStride == 0 &&
                          (g - kDmaStep0) / kDmaStride < G::XPPW) {
                constexpr int j = (g - kDmaStep0) / kDmaStride;
                if constexpr (j % 4 == 0) blk = halo_block(hn, lane, zl, j / 4);
                halo_piece(hn, blk, lds, dw, j);
            }
            if constexpr (g >= 40 && (g - 40) % 7 == 0 && (g - 40) / 7 < NCG * NA) {
                constexpr int j = (g - 40) / 7;
                epilogue(j / NCG, j % NCG, accA[j / NCG][j % NCG]);
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        TB64_STAMP(k, 1);
#pragma unroll
        for (int t = 0; t < NB; t++)
#pragma unroll
            for (int ci = 0; ci < NCG; ci++) epilogue(NA + t, ci, accB[t][ci]);
        TB64_STAMP(k, 2);
        // the next tile's halo has landed (only this phase's 2 x 6 output stores, all issued
        // after the last DMA piece, may still be in flight)
        __builtin_amdgcn_s_waitcnt(wait_vm(2 * G::F2));
        TB64_STAMP(k, 3);
        barrier();
    }
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    TB64_STAMP_FLUSH();
}

template <bool ST>
__global__ __launch_bounds__(256, 1) void tblock64_kernel(TB64Params p) {
    using G = B64;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this workgroup's crops: a balanced contiguous range, walked tile by tile top to bottom
    const int nb = gridDim.x, b = blockIdx.x;
    const int crop0 = (int)(((long)p.N * b) / nb), crop1 = (int)(((long)p.N * (b + 1)) / nb);
    const int n_items = ST ? (b < p.n_tiles ? (p.n_tiles - 1 - b) / nb + 1 : 0) : (crop1 - crop0) * G::TILES_H;
    if (n_items == 0) return;  // whole workgroup: uniform
    // the intermediate's pad and leading slots stay zero for the launch
    for (int i = tid; i < 2 * G::MBYTES / 16; i += 256)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    if (tid < 128) reinterpret_cast<float*>(lds + G::BOFF)[tid] = tid < 64 ? p.b1[tid] : p.b2[tid - 64];
    __builtin_amdgcn_s_waitcnt(kWaitAll);
    if (wave < 2)
        conv1_role<ST>(p, lds, wave, lane, n_items, crop0);
    else
        conv2_role<ST>(p, lds, wave - 2, lane, n_items, p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8, crop0);
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
        MVP_HIP(hipFuncSetAttribute((const void*)tblock64_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        MVP_HIP(hipFuncSetAttribute((const void*)tblock64_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (g_tb64_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_tb64_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long tiles = (long)N * G::TILES_H;
    MVP_REQUIRE(tiles < (1L << 30), "tblock64: too many tiles");
    // contiguous crop ranges (conv1 reuses rows across a crop's tiles) from one crop per CU;
    // smaller batches: tiles strided over every CU, every tile computing all 10 rows
    TB64Params p{x, w1, b1, w2, b2, y, conv_zero_region(), N, (int)tiles};
    if (crop_ranges_balanced(N, g_tb64_cus))
        hipLaunchKernelGGL(tblock64_kernel<false>, dim3(std::min(N, g_tb64_cus)), dim3(256), G::LDS, s, p);
    else
        hipLaunchKernelGGL(tblock64_kernel<true>, dim3((int)std::min<long>(tiles, g_tb64_cus)), dim3(256), G::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
