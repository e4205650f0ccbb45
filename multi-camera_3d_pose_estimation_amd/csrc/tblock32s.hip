// Streaming fused HRNet BasicBlock on the 32-channel 64x48 branch plane (gfx950):
//   y = relu( conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x )
// for HRNet-W32's 32 BasicBlocks on branch 0.  The block is HBM-bound: at 1,024 crops its
// 201 MB input and 201 MB output need ~67 us at 6 TB/s against ~46 us of MFMA work.  The
// tile kernel (tblock.hip) re-reads a 2-row halo per 16-row tile and can overlap the next
// tile's DMA only with conv2 (one input buffer), so its DMA waits are exposed.  Here:
//
// * each workgroup (one per CU, 8 waves) walks WHOLE crops top to bottom in strips of 8
//   output rows; the input arrives row by row into a 30-row LDS ring (each image row is
//   fetched from HBM exactly once; the ring holds every row a phase touches, so a row's DMA
//   never waits on its readers);
// * warp-specialised phases (one barrier each): waves 0-3 run conv1 of strip k (10
//   intermediate rows = conv2's halo, bias + ReLU + bf16 into a double-buffered LDS image;
//   rows outside the image = 0 = conv2's padding), waves 4-7 run conv2 of strip k-1 (+ b2
//   + the residual from the input ring) after one burst of row DMAs for strip k+1; the
//   ReLU / store epilogue of conv2 runs at the start of the next phase, beside conv1's
//   MFMAs.  Each
//   SIMD hosts one wave of each role, so its MFMA pipe always has two independent streams;
//   every wave keeps its conv's 32 couts x 288 K in 72 VGPRs for the launch.
//
// LDS images are plane-major (4 planes of 8 channels, 16-B slots) with a row pitch of 49
// slots (the 49th is zero: x = 48, and x = -1 of the next row; one leading zero slot per
// plane), so a tap is a constant offset; the ring's rows wrap, so conv1 keeps one base
// register per tap row.  Fragments are two 16-pixel row runs (conflict-free ds_read_b128).
// MFMA sequence (bias start, k-step = (tap, 16-channel half)) and epilogues are those of
// tblock32_kernel: the result is bit-identical to it.
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

struct S32 {
    static constexpr int H = 64, W = 48, TH = 8, STRIPS = H / TH;
    static constexpr int RS = W + 1;                 // row pitch (slots)
    static constexpr int VR = H + 4;                 // virtual rows per crop: 2 zero, 64 image, 2 zero
    static constexpr int NR = 30;                    // input ring rows (widest live span: crop boundaries)
    static constexpr int PL = (1 + NR * RS) * 16;    // one input plane: leading zero slot + ring
    static constexpr int XBYTES = 4 * PL;
    static constexpr int MR = TH + 2;                // intermediate rows per strip
    static constexpr int MPL = (1 + MR * RS) * 16;   // one intermediate plane
    static constexpr int MBYTES = 4 * MPL;
    static constexpr int MOFF = XBYTES;
    static constexpr int BOFF = MOFF + 2 * MBYTES;   // b1 | b2 (f32)
    static constexpr int LDS = BOFF + 2 * 32 * 4;
    static constexpr int F1 = MR * W / 32;           // 15 conv1 fragments per strip
    static constexpr int F2 = TH * W / 32;           // 12 conv2 fragments per strip
    static constexpr int NF1 = 4, NF2 = 3;           // fragments per wave (conv1 wave 3: one pad fragment)
    static constexpr int KS = 18;                    // k-steps: 9 taps x 2 halves of 16 channels
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(2 * PL + 2 * 16 < 65536 && 2 * MPL + (2 * RS + 2) * 16 < 65536, "ds_read offset range");
    static_assert(F1 <= 4 * NF1 && F2 == 4 * NF2, "fragment split");
};

constexpr int wait_vm(int n) { return ((n >> 4) << 14) | 0x0F70 | (n & 15); }
constexpr int kWaitLgkm0 = 0xC07F;
constexpr int kWaitAll = 0x0070;

struct S32Params {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y;
    const uint16_t* zero;
    int N;
#ifdef TB32S_STAMPS
    unsigned long long* stamps;  // [block][wave][phase < 16][4] s_memtime (tools/s32_stamps.hip)
#endif
};

#ifdef TB32S_STAMPS
#define S32_STAMP(k, i)                                                                                      \
    do {                                                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                         \
        if ((k) < 16 && (threadIdx.x & 63) == 0)                                                             \
            p.stamps[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + (k)) * 4 + (i)] = t_;                    \
    } while (0)
#else
#define S32_STAMP(k, i) \
    do {                \
    } while (0)
#endif

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

// A fragments of one conv for lane (r32, h): cout row_cout(r32), k-step s = (tap s/2, half
// s%2): input channels 16 (s%2) + 8h .. +7 (tblock32_kernel's weight slot order).
__device__ __forceinline__ void load_weights(const uint16_t* __restrict__ w, int r32, int h, bf16x8 (&wa)[S32::KS]) {
    const int cout = row_cout(r32);
#pragma unroll
    for (int s = 0; s < S32::KS; s++)
        wa[s] = *reinterpret_cast<const bf16x8*>(w + (cout * 9 + (s >> 1)) * 32 + (s & 1) * 16 + 8 * h);
}

// The accumulators start at the lane's 16 biases (couts 16h .. 16h+15) from LDS.
__device__ __forceinline__ f32x16 bias_acc(const uint8_t* lds, int conv, int h) {
    const float4* b = reinterpret_cast<const float4*>(lds + S32::BOFF + (32 * conv + 16 * h) * 4);
    f32x16 r;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float4 q = b[j];
        r[4 * j] = q.x;
        r[4 * j + 1] = q.y;
        r[4 * j + 2] = q.z;
        r[4 * j + 3] = q.w;
    }
    return r;
}

// Strip g of this workgroup's crop range: crop-local index, strip in the crop.
struct Strip {
    int cl, s;
};
__device__ __forceinline__ Strip strip_of(int g) { return Strip{g >> 3, g & 7}; }
__device__ __forceinline__ int ring_row(int v) { return v % S32::NR; }

// Rows the DMA brings in for strip g: virtual rows [v0, v0 + n) of its crop (v = image row + 2).
__device__ __forceinline__ void strip_rows(int g, int& v0, int& n) {
    const Strip st = strip_of(g);
    const int base = st.cl * S32::VR;
    if (st.s == 0) {
        v0 = base;
        n = 12;
    } else {
        v0 = base + 8 * st.s + 4;
        n = 8;
    }
}

// One ring row (virtual row v of crop-local cl, plane q): lanes 0-47 the 48 pixels' 16-B
// plane chunk, lane 48 the pad slot (zero); rows outside the image read the zero region.
__device__ __forceinline__ void dma_row(const S32Params& p, uint8_t* lds, int crop, int cl, int v, int q, int lane,
                                        const uint16_t* zl) {
    using G = S32;
    const int ir = v - cl * G::VR - 2;
    const bool in = (unsigned)ir < (unsigned)G::H && lane < G::W;
    const uint16_t* src = in ? p.x + (((long)crop * G::H + ir) * G::W + lane) * 32 + q * 8 : zl;
    if (lane < G::RS) glds16(src, lds + q * G::PL + (1 + ring_row(v) * G::RS) * 16);
}

// Rows [i0, i1) of strip g's row load (strip_rows), plane q, as one burst of row DMAs.
__device__ __forceinline__ void dma_strip_rows(const S32Params& p, uint8_t* lds, int crop0, int g, int i0, int i1,
                                               int q, int lane, const uint16_t* zl) {
    using G = S32;
    int v0, n;
    strip_rows(g, v0, n);
    const int cl = strip_of(g).cl;
    const int ir0 = v0 - cl * G::VR - 2;
    const long base = (((long)(crop0 + cl) * G::H + ir0) * G::W + lane) * 32 + q * 8;
    int rr = ring_row(v0 + i0);
#ifdef TB32S_DIAG_NO_DMA  // stamps harness only: timing without the row DMAs (stale rows)
    if (g > 1) return;
#endif
    for (int i = i0; i < min(i1, n); i++) {
        const bool in = (unsigned)(ir0 + i) < (unsigned)G::H && lane < G::W;
        if (lane < G::RS) glds16(in ? p.x + base + (long)i * G::W * 32 : zl, lds + q * G::PL + (1 + rr * G::RS) * 16);
        rr = rr + 1 == G::NR ? 0 : rr + 1;
    }
}

// B fragments prefetched this many k-steps ahead (conv1 / conv2 waves)
#ifndef TB32S_PF1
#define TB32S_PF1 4
#endif
#ifndef TB32S_PF2
#define TB32S_PF2 3
#endif
// Row DMAs of the next strip: the conv2 waves issue rows [0, kDmaSplit) of its load, the
// conv1 waves the rest (each a burst at the start of its phase).  8: a strip's 8 new rows all
// on the conv2 waves, so each SIMD's conv1 wave starts its MFMAs at once instead of both waves
// of the SIMD issuing DMA first; only the 12-row load of a crop's first strip gives its last 4
// rows to the conv1 waves (round 4, same box: the former 4 / 8 split 131.8 us per block, all on
// the conv1 waves 141.2, all 12 on the conv2 waves 121.5; with conv1's row reuse, 12: 116.5,
// 8: 112.4 -- profiles/r04_dma_split_ab.txt)
constexpr int kDmaSplit = 8;

// conv1 waves (j = 0..3).  The first strip of a crop: fragments j, j+4, j+8, j+12 of the
// strip's 10 intermediate rows (image rows 8s - 1 .. 8s + 8; one pad fragment).  Later strips:
// rows 0-1 are the previous strip's rows 8-9, copied from the other intermediate buffer (wave j
// copies plane j), and only rows 2-9 are computed: fragments 3 + j, 7 + j, 11 + j (12 instead of
// 15 + 1 pad; 54 instead of 72 MFMAs per wave).  Same MFMA sequence per row: bit-identical.
// (Round 4: 123.0 -> 114.8 us per block same-box, profiles/r04_tblock64_rowreuse_ab.txt.)
__device__ __forceinline__ void conv1_role(const S32Params& p, uint8_t* lds, int j, int lane, int n_strips, int crop0,
                                           const uint16_t* zl) {
    using G = S32;
    constexpr int RS = G::RS, NF = G::NF1;
    constexpr int kPF = TB32S_PF1;
    const int h = lane >> 5, r32 = lane & 31;
    bf16x8 wa[G::KS];
    load_weights(p.w1, r32, h, wa);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    // full set (first strip of a crop): NF fragments, the last a pad on wave 3; reuse set: 3
    int pi[NF], px[NF], pir[3], pxr[3];
    bool pad[NF], padr[3] = {false, false, false};
#pragma unroll
    for (int t = 0; t < NF; t++) {
        int f = j + 4 * t;
        pad[t] = f >= G::F1;
        if (pad[t]) f = j;  // a duplicate of the wave's first fragment: computed, never stored
        const int pp = frag_pixel<G::W, G::MR, 1>(f, r32);
        pi[t] = pp / G::W;
        px[t] = pp - pi[t] * G::W;
    }
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const int pp = frag_pixel<G::W, G::MR, 1>(3 + j + 4 * t, r32);
        pir[t] = pp / G::W;
        pxr[t] = pp - pir[t] * G::W;
    }
    // one strip's conv1: NA fragments in half A, NB in half B (half A's epilogues run in the
    // shadow of half B's MFMAs; only half B's is exposed)
    auto strip_body = [&](auto na_tag, auto nb_tag, const int* fpi, const int* fpx, const bool* fpad, int k,
                          const Strip& st) {
        constexpr int NA = decltype(na_tag)::value, NB = decltype(nb_tag)::value, NT = NA + NB;
        constexpr int NM = NA > NB ? NA : NB;
        const int v0 = st.cl * G::VR + 8 * st.s;  // virtual row of intermediate row 0's tap row 0
        int bv[NT][3];
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int dy = 0; dy < 3; dy++)
                bv[t][dy] = h * G::PL + (ring_row(v0 + fpi[t] + dy) * RS + fpx[t]) * 16;
        constexpr int NS = (NB > 0 ? 2 : 1) * G::KS;
        f32x16 accA[NA], accB[NB > 0 ? NB : 1];
        accA[0] = bias_acc(lds, 0, h);
#pragma unroll
        for (int t = 1; t < NA; t++) accA[t] = accA[0];
#pragma unroll
        for (int t = 0; t < NB; t++) accB[t] = accA[0];
        uint8_t* mb = lds + G::MOFF + (k & 1) * G::MBYTES;
        auto epilogue = [&](int t, const f32x16& a) {
            if (fpad[t]) return;
            // intermediate row pi = image row 8s - 1 + pi: rows outside are conv2's zero padding
            const bool live = (unsigned)(8 * st.s - 1 + fpi[t]) < (unsigned)G::H;
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) o[e] = live ? pack_bf16x2(relu1(a[2 * e]), relu1(a[2 * e + 1])) : 0u;
            uint8_t* d = mb + (2 * h * G::MPL / 16 + 1 + fpi[t] * RS + fpx[t]) * 16;
            *reinterpret_cast<uint4*>(d) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(d + G::MPL) = uint4{o[4], o[5], o[6], o[7]};
        };
        bf16x8 fb[kPF + 1][NM];
        auto load = [&](auto Gs) {
            constexpr int g = Gs, s = g % G::KS, hb = g / G::KS, t0 = hb * NA, nt = hb ? NB : NA;
            constexpr int tap = s >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int t = 0; t < nt; t++)
                fb[g % (kPF + 1)][t] =
                    *reinterpret_cast<const bf16x8*>(lds + bv[t0 + t][dy] + (2 * ks * (G::PL / 16) + dx) * 16);
        };
        static_for<0, kPF>(load);
        static_for<0, NS>([&](auto Gs) {
            constexpr int g = Gs, s = g % G::KS;
            if constexpr (g + kPF < NS) load(std::integral_constant<int, g + kPF>{});
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g < G::KS) {
#pragma unroll
                for (int t = 0; t < NA; t++)
                    accA[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], fb[g % (kPF + 1)][t], accA[t], 0, 0, 0);
            } else {
#pragma unroll
                for (int t = 0; t < NB; t++)
                    accB[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], fb[g % (kPF + 1)][t], accB[t], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g >= G::KS + 3 && (g - G::KS - 3) % 6 == 0 && (g - G::KS - 3) / 6 < NA)
                epilogue((g - G::KS - 3) / 6, accA[(g - G::KS - 3) / 6]);
            __builtin_amdgcn_sched_barrier(0);
        });
        S32_STAMP(k, 1);
#pragma unroll
        for (int t = 0; t < NB; t++) epilogue(NA + t, accB[t]);
    };
    barrier();  // prologue: strip 0's rows, zeroed images, biases
    for (int k = 0; k <= n_strips; k++) {
        S32_STAMP(k, 0);
        // the upper rows of strip k+1's load (the conv2 waves bring the first kDmaSplit)
        if (k + 1 < n_strips) dma_strip_rows(p, lds, crop0, k + 1, kDmaSplit, 12, j, lane, zl);
        if (k < n_strips) {
            const Strip st = strip_of(k);
            if (st.s == 0) {
                strip_body(std::integral_constant<int, NF / 2>{}, std::integral_constant<int, NF / 2>{}, pi, px, pad, k,
                           st);
            } else {
                // rows 0-1 = the previous strip's rows 8-9 (plane j, pad slots included)
                const uint8_t* mp = lds + G::MOFF + ((k - 1) & 1) * G::MBYTES + j * G::MPL + 16;
                uint8_t* mc = lds + G::MOFF + (k & 1) * G::MBYTES + j * G::MPL + 16;
                for (int i = lane; i < 2 * RS; i += 64)
                    *reinterpret_cast<uint4*>(mc + i * 16) = *reinterpret_cast<const uint4*>(mp + (8 * RS + i) * 16);
                strip_body(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{}, pir, pxr, padr, k, st);
            }
            __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
            S32_STAMP(k, 2);
        }
        __builtin_amdgcn_s_waitcnt(wait_vm(0));  // this wave's rows of strip k+1 have landed
        barrier();
    }
}

// conv2 waves (j = 0..3): in phase k, the DMA of strip k+1's rows (plane j of each row) and
// conv2 of strip k-1 (fragments j, j+4, j+8) + b2 + residual + ReLU -> y.
__device__ __forceinline__ void conv2_role(const S32Params& p, uint8_t* lds, int j, int lane, int n_strips,
                                           int crop0, const uint16_t* zl) {
    using G = S32;
    constexpr int RS = G::RS, NF = G::NF2;
    constexpr int kPF = TB32S_PF2;
    const int h = lane >> 5, r32 = lane & 31;
    bf16x8 wa[G::KS];
    load_weights(p.w2, r32, h, wa);
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
    int pr[NF], px[NF];
#pragma unroll
    for (int t = 0; t < NF; t++) {
        const int pp = frag_pixel<G::W, G::TH, 1>(j + 4 * t, r32);
        pr[t] = pp / G::W;
        px[t] = pp - pr[t] * G::W;
    }
    {  // prologue: strip 0's 12 rows
        int v0, n;
        strip_rows(0, v0, n);
        for (int i = 0; i < n; i++) dma_row(p, lds, crop0, 0, v0 + i, j, lane, zl);
        __builtin_amdgcn_s_waitcnt(wait_vm(0));
    }
    barrier();
    // C2(k-1)'s accumulators and residual live across the barrier: its epilogue (residual
    // add, ReLU, bf16, stores) runs at the start of phase k+1, beside the conv1 waves' MFMAs,
    // instead of on the phase's critical path
    f32x16 acc[NF];
    uint4 rv[NF][2];
    long pix_prev = 0;
    auto epilogue = [&]() {
#pragma unroll
        for (int t = 0; t < NF; t++) {
            uint32_t o[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint4 rr = rv[t][e >> 2];
                const uint32_t u = (e & 3) == 0 ? rr.x : (e & 3) == 1 ? rr.y : (e & 3) == 2 ? rr.z : rr.w;
                o[e] = pack_bf16x2(relu1(acc[t][2 * e] + lo_bf16(u)), relu1(acc[t][2 * e + 1] + hi_bf16(u)));
            }
            uint16_t* yp = p.y + (pix_prev + pr[t] * G::W + px[t]) * 32 + 16 * h;
#ifdef TB32S_DIAG_NO_STORE  // stamps harness only: timing without the output stores (wrong results)
            if ((o[0] ^ o[3] ^ o[5]) == 0x12345678u)
#endif
            {
#ifdef TB32S_NT_STORE  // A/B: non-temporal output stores
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<u32x4*>(yp));
                __builtin_nontemporal_store(u32x4{o[4], o[5], o[6], o[7]}, reinterpret_cast<u32x4*>(yp + 8));
#else
                *reinterpret_cast<uint4*>(yp) = uint4{o[0], o[1], o[2], o[3]};
                *reinterpret_cast<uint4*>(yp + 8) = uint4{o[4], o[5], o[6], o[7]};
#endif
            }
        }
    };
    for (int k = 0; k <= n_strips; k++) {
        S32_STAMP(k, 0);
        // this phase's DMA: strip k+1's rows (12 or 8; none past the last strip), one burst
        // ahead of everything else: the ring rows it fills are read by no one in this phase,
        // and row DMAs interleaved with the k-steps made the compiler drain every LDS read
        // (lgkmcnt(0)) at each step (measured: conv2 loop 7.0k ticks for 1.7k of MFMA)
        if (k + 1 < n_strips) dma_strip_rows(p, lds, crop0, k + 1, 0, kDmaSplit, j, lane, zl);
        S32_STAMP(k, 1);
        if (k >= 2) epilogue();  // C2(k-2): its stores are younger than this phase's DMA
        S32_STAMP(k, 2);
        if (k >= 1) {
            const Strip st = strip_of(k - 1);
            const uint8_t* mb = lds + G::MOFF + ((k - 1) & 1) * G::MBYTES;
            int bv[NF];
#pragma unroll
            for (int t = 0; t < NF; t++) {
                bv[t] = (int)(mb - lds) + h * G::MPL + (pr[t] * RS + px[t]) * 16;
                // residual: image row 8s + pr = virtual row 8s + pr + 2, planes 2h and 2h+1
                const int rr = ring_row(st.cl * G::VR + 8 * st.s + pr[t] + 2);
                const uint8_t* rb = lds + (2 * h * G::PL / 16 + 1 + rr * RS + px[t]) * 16;
                rv[t][0] = *reinterpret_cast<const uint4*>(rb);
                rv[t][1] = *reinterpret_cast<const uint4*>(rb + G::PL);
            }
            acc[0] = bias_acc(lds, 1, h);
#pragma unroll
            for (int t = 1; t < NF; t++) acc[t] = acc[0];
            bf16x8 fb[kPF + 1][NF];
            auto load = [&](auto Ss) {
                constexpr int s = Ss, tap = s >> 1, ks = s & 1, dy = tap / 3, dx = tap % 3;
#pragma unroll
                for (int t = 0; t < NF; t++)
                    fb[s % (kPF + 1)][t] = *reinterpret_cast<const bf16x8*>(
                        lds + bv[t] + (2 * ks * (G::MPL / 16) + dy * RS + dx) * 16);
            };
            static_for<0, kPF>(load);
            static_for<0, G::KS>([&](auto Ss) {
                constexpr int s = Ss;
                if constexpr (s + kPF < G::KS) load(std::integral_constant<int, s + kPF>{});
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < NF; t++)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], fb[s % (kPF + 1)][t], acc[t], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            });
            pix_prev = ((long)(crop0 + st.cl) * G::H + 8 * st.s) * G::W;
        }
        S32_STAMP(k, 3);
        // the next strip's rows have landed (only this phase's 2 NF output stores may be younger)
        if (k >= 2)
            __builtin_amdgcn_s_waitcnt(wait_vm(2 * NF));
        else
            __builtin_amdgcn_s_waitcnt(wait_vm(0));
        barrier();
    }
    epilogue();  // the last strip's C2
    __builtin_amdgcn_s_waitcnt(wait_vm(0));
}

__global__ __launch_bounds__(512, 1) void tblock32s_kernel(S32Params p) {
    using G = S32;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this workgroup's crops: a balanced contiguous range
    const int nb = gridDim.x, b = blockIdx.x;
    const int crop0 = (int)(((long)p.N * b) / nb), crop1 = (int)(((long)p.N * (b + 1)) / nb);
    const int n_strips = (crop1 - crop0) * G::STRIPS;
    if (n_strips == 0) return;  // whole workgroup: uniform
    // zero: the input ring's leading slots, the intermediate images (pad slots stay zero)
    if (tid < 4) *reinterpret_cast<uint4*>(lds + tid * G::PL) = uint4{0u, 0u, 0u, 0u};
    for (int i = tid; i < 2 * G::MBYTES / 16; i += 512)
        *reinterpret_cast<uint4*>(lds + G::MOFF + i * 16) = uint4{0u, 0u, 0u, 0u};
    if (tid < 64) reinterpret_cast<float*>(lds + G::BOFF)[tid] = tid < 32 ? p.b1[tid] : p.b2[tid - 32];
    __builtin_amdgcn_s_waitcnt(kWaitAll);
#ifndef TB32S_PRIO2
#define TB32S_PRIO2 0
#endif
    // conv2 waves carry the phase's critical path (DMA burst, stores, then MFMAs): optional
    // static issue priority over the conv1 wave on the same SIMD
    if (TB32S_PRIO2 > 0 && wave >= 4) __builtin_amdgcn_s_setprio(TB32S_PRIO2);
    if (wave < 4)
        conv1_role(p, lds, wave, lane, n_strips, crop0, p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8);
    else
        conv2_role(p, lds, wave - 4, lane, n_strips, crop0, p.zero + ((wave * 64 + lane) & (kZeroSlots - 1)) * 8);
}

int g_s32_cus = 0;

}  // namespace

bool launch_tblock32s(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                      uint16_t* y, int N, int H, int W, hipStream_t s) {
    using G = S32;
    if (H != G::H || W != G::W) return false;
    const char* e = getenv("MVPOSE_NO_TBLOCK32S");  // A/B and tests: the tile kernel (tblock.hip)
    const char* e2 = getenv("MVPOSE_NO_TBLOCK");    // tests: no 32x32x16 block kernel at all
    if ((e && e[0] == '1') || (e2 && e2[0] == '1')) return false;
    if (N == 0) return true;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)tblock32s_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (g_s32_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_s32_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (!crop_ranges_balanced(N, g_s32_cus)) return false;  // small / ragged batch: the tile kernel
    MVP_REQUIRE(N < (1 << 24), "tblock32s: too many crops");
    S32Params p{x, w1, b1, w2, b2, y, conv_zero_region(), N};
    const int grid = std::min(N, g_s32_cus);
    hipLaunchKernelGGL(tblock32s_kernel, dim3(grid), dim3(512), G::LDS, s, p);
    MVP_HIP(hipGetLastError());
    return true;
}

}  // namespace mvp
