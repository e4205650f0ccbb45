// 1x1 convolutions (HRNet Bottleneck / downsample / fuse-layer projections) for gfx950.
//
// A 1x1 conv has no spatial reuse, so staging the input through LDS buys nothing:
// each lane's B fragment (8 consecutive channels of one pixel, NHWC) is one 16-B
// global load straight into registers.  The block's weight slice ([chunk][q][cout]
// 16-B slots, BM couts x Cin) is DMA'd into LDS once; waves then run independently
// over 16*PTW-pixel units with no barriers: loads of B (+ residual) -> MFMA
// (v_mfma_f32_16x16x32_bf16, A fragments from LDS, each reused by PTW pixel tiles)
// -> bias [+ residual] [+ ReLU] -> bf16 NHWC stores.  Same MFMA, same K order
// (chunk 0..Cin/32-1) and same epilogue arithmetic as conv_mfma_kernel.  The A
// rows are a permutation of the block's couts, so that each lane group owns BM/4
// consecutive couts of its pixel: residual loads and stores are 16 B per lane
// (the layer1 64->256 projections are memory-bound; 8-B accesses made them
// issue-bound).
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "mvp_common.h"

namespace mvp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}

struct P1x1 {
    const uint16_t* x;
    const uint16_t* w;
    const float* bias;
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* zero;
    long n_pix;
    int Cout, relu;
    // dual input (graph cat-fusion): K chunks [0, kch1) read x (c1 channels per pixel),
    // the rest x2 (c2 channels); single input: x2 = nullptr, c1 = Cin, kch1 = Cin / 32
    const uint16_t* x2;
    int c1, c2, kch1;
};

constexpr int kPTW = 2;  // 16-pixel tiles per wave per unit

template <int BM, int KCH>
__global__ __launch_bounds__(256, 2) void conv1x1_kernel(P1x1 p) {
    constexpr int NCT = BM / 16, CIN = KCH * 32, SLOTS = KCH * 4 * BM;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    __shared__ float4 sbias[BM / 4];
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int co0 = blockIdx.y * BM;
    for (int s0 = wave * 64; s0 < SLOTS; s0 += 256) {
        const int sl = s0 + lane;
        const void* src = p.zero;
        if (sl < SLOTS) {
            const int co = sl % BM, tq = sl / BM;  // tq = chunk * 4 + q
            // A row r of cout tile c holds cout (r>>2)*(BM/4) + 4c + (r&3): output lane
            // group g then owns the BM/4 consecutive couts g*(BM/4) .. of its pixel
            const int c = co >> 4, r = co & 15;
            src = p.w + (size_t)(co0 + (r >> 2) * (BM / 4) + c * 4 + (r & 3)) * CIN + tq * 8;
        }
        glds16(src, lds + s0 * 16);
    }
    if (tid < BM / 4) sbias[tid] = reinterpret_cast<const float4*>(p.bias + co0)[tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const long n_units = (p.n_pix + 16 * kPTW - 1) / (16 * kPTW);
    for (long u = (long)blockIdx.x * 4 + wave; u < n_units; u += (long)gridDim.x * 4) {
        long pix[kPTW];
        bool valid[kPTW];
        bf16x8 b[kPTW][KCH];
#pragma unroll
        for (int i = 0; i < kPTW; i++) {
            const long pp = u * 16 * kPTW + i * 16 + (lane & 15);
            valid[i] = pp < p.n_pix;
            pix[i] = valid[i] ? pp : p.n_pix - 1;
            const uint16_t* src = p.x + pix[i] * p.c1 + g * 8;
            const uint16_t* src2 = p.x2 ? p.x2 + pix[i] * p.c2 + g * 8 - p.kch1 * 32 : src;
#pragma unroll
            for (int ch = 0; ch < KCH; ch++)
                b[i][ch] = *reinterpret_cast<const bf16x8*>((ch < p.kch1 ? src : src2) + ch * 32);
        }
        // residual: the lane's BM/4 consecutive couts, 16 B per load
        constexpr int RQ = BM / 32;  // uint4 per lane per pixel tile
        uint4 rv[kPTW][RQ];
        const int cog = co0 + g * (BM / 4);
        const bool co_ok = cog < p.Cout;
#pragma unroll
        for (int i = 0; i < kPTW; i++) {
            const uint16_t* src = (p.res && co_ok) ? p.res + pix[i] * p.Cout + cog : p.zero + lane * (BM / 4);
#pragma unroll
            for (int q = 0; q < RQ; q++) rv[i][q] = *reinterpret_cast<const uint4*>(src + q * 8);
        }
        f32x4 acc[kPTW][NCT];
#pragma unroll
        for (int i = 0; i < kPTW; i++)
#pragma unroll
            for (int c = 0; c < NCT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ch = 0; ch < KCH; ch++)
#pragma unroll
            for (int c = 0; c < NCT; c++) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + ((ch * 4 + g) * BM + c * 16 + (lane & 15)) * 16);
#pragma unroll
                for (int i = 0; i < kPTW; i++)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[i][ch], acc[i][c], 0, 0, 0);
            }
#pragma unroll
        for (int i = 0; i < kPTW; i++) {
            uint32_t o[2 * NCT];
#pragma unroll
            for (int c = 0; c < NCT; c++) {
                const float4 bb = sbias[g * (BM / 16) + c];
                float v[4] = {acc[i][c][0] + bb.x, acc[i][c][1] + bb.y, acc[i][c][2] + bb.z, acc[i][c][3] + bb.w};
                const uint4 r4 = rv[i][c >> 1];
                const uint32_t r0 = (c & 1) ? r4.z : r4.x, r1 = (c & 1) ? r4.w : r4.y;
                v[0] += bf16_to_f32(r0 & 0xffff);
                v[1] += bf16_to_f32(r0 >> 16);
                v[2] += bf16_to_f32(r1 & 0xffff);
                v[3] += bf16_to_f32(r1 >> 16);
                if (p.relu) {
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
                }
                o[2 * c] = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
                o[2 * c + 1] = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
            }
            if (valid[i] && co_ok) {
                uint16_t* yrow = p.y + pix[i] * p.Cout + cog;
#pragma unroll
                for (int q = 0; q < RQ; q++)
                    *reinterpret_cast<uint4*>(yrow + q * 8) = uint4{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
            }
        }
    }
}

// ------------------------------------------------------------ bottleneck join
// Layer1 of HRNet-W32 alternates conv3 (64 -> 256, + residual, ReLU) and the next
// block's conv1 (256 -> 64, ReLU) at 64x48: the 256-ch tensor (1.6 GB per 1024
// crops) was written by one launch and read straight back by the next.  Here one
// wave computes all 256 couts of 16 pixels in two halves of 128 (A rows permuted so
// that in half h lane group g holds couts 128h + 32g .. + 31 of its pixel), stores
// them (through a per-wave LDS staging block, as whole 256-B runs) and feeds the same
// bf16 values to the second GEMM as B fragments without any lane exchange: the second
// GEMM's K order is permuted to match — K chunk j, lane group g covers channels
// 128 (j >> 2) + 32g + 8 (j & 3) .. + 7 — by the order the W2 slots are DMA'd into
// LDS.  The residual is loaded coalesced and transposed through the same block.  y is
// rounded to bf16 before the second GEMM, as in the unfused graph; only the f32
// summation order of the second GEMM differs.
struct PPair {
    const uint16_t* x;
    const uint16_t* x2;
    int c1, c2, kch1;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y2;
    const uint16_t* zero;
    long n_pix;
};

// threads per workgroup (one workgroup per CU, 2 waves per SIMD): 12-wave workgroups
// (3 per SIMD) measured slower, 1067 vs 1018 us per join
template <int KCH>
constexpr int pair_threads() { return 512; }

// KCH: K chunks of the first GEMM (2: 64 ch, 4: the cat-fused 64 + 64); RES: conv3 adds a
// residual (the cat-fused join has none: its downsample is folded into K); LA: units of
// load look-ahead per wave.  This kernel is bound by the bytes each wave keeps in flight
// (8 waves per CU): with one unit ahead the cat-fused join had 4 KB per wave in flight
// and moved 2.5 TB/s.
// SECOND = false: conv3 alone (layer1's last block, whose output goes to transition1),
// same 256-cout waves and staged stores, no second GEMM.
template <int KCH, bool RES, int LA, bool SECOND = true>
__global__ __launch_bounds__(pair_threads<KCH>(), 1) void conv1x1_pair_kernel(PPair p) {
    constexpr int kPairThreads = pair_threads<KCH>();
    constexpr int BM = 256, NCT = BM / 16, CIN = KCH * 32;
    constexpr int S1 = KCH * 4 * BM;            // expand weight slots [chunk][q][row]
    constexpr int S2 = SECOND ? 8 * 4 * 64 : 0;  // reduce weight slots [chunk][q][row]
    constexpr int R = LA + 1;         // register ring of units (current + LA ahead)
    constexpr int NRQ = RES ? 8 : 1;  // residual uint4 per lane per unit
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    __shared__ float4 sb1[BM / 4];
    __shared__ float4 sb2[16];
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int NWAVES = kPairThreads / 64;
    for (int s0 = wave * 64; s0 < S1 + S2; s0 += kPairThreads) {
        const int sl = s0 + lane;
        const void* src = p.zero;
        if (sl < S1) {
            // A row r of cout tile c holds cout 128 (c >> 3) + 32 (r >> 2) + 4 (c & 7) + (r & 3):
            // in half h (tiles 8h .. 8h + 7) lane group g owns couts 128h + 32g .. + 31
            const int co = sl % BM, tq = sl / BM;
            const int c = co >> 4, r = co & 15;
            src = p.w1 + (size_t)(128 * (c >> 3) + 32 * (r >> 2) + 4 * (c & 7) + (r & 3)) * CIN + tq * 8;
        } else if (sl < S1 + S2) {
            // second GEMM K chunk j, lane group q: channels 128 (j >> 2) + 32 q + 8 (j & 3)
            const int s2 = sl - S1, co = s2 % 64, tq = s2 / 64;  // tq = chunk j * 4 + q
            const int c = co >> 4, r = co & 15, j = tq >> 2, q = tq & 3;
            src = p.w2 + (size_t)((r >> 2) * 16 + c * 4 + (r & 3)) * 256 + 128 * (j >> 2) + 32 * q + 8 * (j & 3);
        }
        glds16(src, lds + s0 * 16);
    }
    if (tid < BM / 4) sb1[tid] = reinterpret_cast<const float4*>(p.b1)[tid];
    if (SECOND && tid < 16) sb2[tid] = reinterpret_cast<const float4*>(p.b2)[tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t* lds2 = lds + S1 * 16;
    uint8_t* stg = lds + (S1 + S2) * 16 + wave * 4096;  // this wave's 4 KiB y staging block

    const long n_units = (p.n_pix + 15) / 16;
    const long ustep = (long)gridDim.x * NWAVES;
    // software pipeline: unit u + LA's input and residual loads are issued before unit u's
    // MFMAs; ring slot of unit u0 + i * ustep is i % R (all indices compile-time)
    struct UnitRegs {
        bf16x8 b[KCH];
        uint4 r[NRQ];
    };
    UnitRegs ring[R];
    auto load_unit = [&](long u, UnitRegs& ur) {
        bf16x8 (&bn)[KCH] = ur.b;
        uint4 (&rn)[NRQ] = ur.r;
        const long pp = u * 16 + (lane & 15);
        const long pix = pp < p.n_pix ? pp : p.n_pix - 1;
        const uint16_t* src = p.x + pix * p.c1 + g * 8;
        const uint16_t* src2 = p.x2 ? p.x2 + pix * p.c2 + g * 8 - p.kch1 * 32 : src;
#pragma unroll
        for (int ch = 0; ch < KCH; ch++)
            bn[ch] = *reinterpret_cast<const bf16x8*>((ch < p.kch1 ? src : src2) + ch * 32);
        if (RES) {  // coalesced: load 4h + i = pixels 4i .. 4i + 3, couts 128h .. 128h + 127
            const long pr0 = u * 16 + (lane >> 4);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const long pr = pr0 + 4 * (q & 3);
                const long pc = pr < p.n_pix ? pr : p.n_pix - 1;
                rn[q] = *reinterpret_cast<const uint4*>(p.res + pc * BM + 128 * (q >> 2) + (lane & 15) * 8);
            }
        }
    };
    // the unit's registers by value: two inlined copies merged by the compiler must select
    // values, not a pointer into the ring (that sent the ring to scratch)
    auto process = [&](long u, const UnitRegs cur) {
        const bf16x8(&b)[KCH] = cur.b;
        const uint4(&rr)[NRQ] = cur.r;
        f32x4 acc2[4];
#pragma unroll
        for (int c = 0; c < 4; c++) acc2[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        // two halves of 8 cout tiles: lane group g's couts 128h + 32g .. + 31, i.e. the
        // second GEMM's K chunks j = 4h .. 4h + 3 (register pressure: one half of the
        // accumulators and packed outputs live at a time)
        uint4 rhalf[RES ? 4 : 1];
        if (RES) {
#pragma unroll
            for (int i = 0; i < 4; i++) rhalf[i] = rr[i];
        }
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            // residual of half h: through the staging block into the owner layout (the
            // inverse of the y staging below; lane group g gets couts 128h + 32g .. + 31)
            uint4 rv[NRQ > 1 ? 4 : 1];
            if (RES) {
                const int k = lane & 15;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int pr = 4 * i + (lane >> 4);
                    *reinterpret_cast<uint4*>(stg + pr * 256 + ((k ^ pr) << 4)) = rhalf[i];
                }
                const int px = lane & 15;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    rv[q] = *reinterpret_cast<const uint4*>(stg + px * 256 + (((4 * g + q) ^ px) << 4));
#pragma unroll
                for (int i = 0; i < 4; i++) rhalf[i] = rr[4 + i];  // the next half's
            }
            f32x4 acc[NCT / 2];
#pragma unroll
            for (int c = 0; c < NCT / 2; c++) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ch = 0; ch < KCH; ch++)
#pragma unroll
                for (int c = 0; c < NCT / 2; c++) {
                    const int ct = h * (NCT / 2) + c;
                    const bf16x8 a =
                        *reinterpret_cast<const bf16x8*>(lds + ((ch * 4 + g) * BM + ct * 16 + (lane & 15)) * 16);
                    acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[ch], acc[c], 0, 0, 0);
                }
            uint32_t o[NCT];
#pragma unroll
            for (int c = 0; c < NCT / 2; c++) {
                const float4 bb = sb1[32 * h + 8 * g + c];
                float v[4] = {acc[c][0] + bb.x, acc[c][1] + bb.y, acc[c][2] + bb.z, acc[c][3] + bb.w};
                if (RES) {
                    const uint4 r4 = rv[c >> 1];
                    const uint32_t r0 = (c & 1) ? r4.z : r4.x, r1 = (c & 1) ? r4.w : r4.y;
                    v[0] += bf16_to_f32(r0 & 0xffff);
                    v[1] += bf16_to_f32(r0 >> 16);
                    v[2] += bf16_to_f32(r1 & 0xffff);
                    v[3] += bf16_to_f32(r1 >> 16);
                }
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
                o[2 * c] = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
                o[2 * c + 1] = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
            }
            // y stores through the wave's LDS staging block: a half is 16 pixels x 128
            // contiguous couts (256 B), so 16 lanes store one pixel's run and an instruction
            // writes 4 whole runs.  Lane-owned 64-B pieces stored directly were 64 separate
            // 16-B requests per instruction (cat-fused join: 1015 us; 64-B runs: 788 us; 599 us
            // for the same bytes lane-contiguous).  Pixel px's run at px * 256, 16-B chunk k
            // (= 4g + q) at slot k ^ px: conflict-free for ds_write_b128 and ds_read_b128.
            {
                const int px = lane & 15;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    *reinterpret_cast<uint4*>(stg + px * 256 + (((4 * g + q) ^ px) << 4)) =
                        uint4{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
                const int k = lane & 15;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int pr = 4 * i + (lane >> 4);
                    const long pq = u * 16 + pr;
                    const uint4 v = *reinterpret_cast<const uint4*>(stg + pr * 256 + ((k ^ pr) << 4));
                    if (pq < p.n_pix) *reinterpret_cast<uint4*>(p.y + pq * BM + 128 * h + k * 8) = v;
                }
            }
            // second GEMM, K chunks j = 4h + jj: this lane group's channels 128h + 32g + 8jj .. +7
#pragma unroll
            for (int jj = 0; jj < (SECOND ? 4 : 0); jj++) {
                const int j = h * 4 + jj;
                union {
                    uint4 u;
                    bf16x8 v;
                } bj;
                bj.u = uint4{o[4 * jj], o[4 * jj + 1], o[4 * jj + 2], o[4 * jj + 3]};
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const bf16x8 a =
                        *reinterpret_cast<const bf16x8*>(lds2 + ((j * 4 + g) * 64 + c * 16 + (lane & 15)) * 16);
                    acc2[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bj.v, acc2[c], 0, 0, 0);
                }
            }
        }
        if (!SECOND) return;
        uint32_t o2[8];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float4 bb = sb2[g * 4 + c];
            const float v0 = fmaxf(acc2[c][0] + bb.x, 0.f), v1 = fmaxf(acc2[c][1] + bb.y, 0.f);
            const float v2 = fmaxf(acc2[c][2] + bb.z, 0.f), v3 = fmaxf(acc2[c][3] + bb.w, 0.f);
            o2[2 * c] = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
            o2[2 * c + 1] = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
        }
        // y2 (64 ch = 128-B pixel rows) through the staging block too: chunk k = 2g + q of
        // pixel px at px * 128 + (k ^ px & 7) * 16; then 8 lanes store one whole row and an
        // instruction 1 KiB of consecutive pixels
        {
            const int px = lane & 15;
            *reinterpret_cast<uint4*>(stg + px * 128 + (((2 * g) ^ px) & 7) * 16) = uint4{o2[0], o2[1], o2[2], o2[3]};
            *reinterpret_cast<uint4*>(stg + px * 128 + (((2 * g + 1) ^ px) & 7) * 16) =
                uint4{o2[4], o2[5], o2[6], o2[7]};
            const int k = lane & 7;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int pr = 8 * i + (lane >> 3);
                const long pq = u * 16 + pr;
                const uint4 v = *reinterpret_cast<const uint4*>(stg + pr * 128 + ((k ^ pr) & 7) * 16);
                if (pq < p.n_pix) *reinterpret_cast<uint4*>(p.y2 + pq * 64 + k * 8) = v;
            }
        }
    };
    const long u0 = (long)blockIdx.x * NWAVES + wave;
#pragma unroll
    for (int i = 0; i < LA; i++)
        if (u0 + i * ustep < n_units) load_unit(u0 + i * ustep, ring[i]);
    for (long u = u0; u < n_units; u += R * ustep) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const long uu = u + r * ustep;
            if (uu < n_units) {  // (no break: the ring indices must stay compile-time)
                const long un = uu + LA * ustep;
                if (un < n_units) load_unit(un, ring[(r + LA) % R]);
                process(uu, ring[r]);
            }
        }
    }
}

// ------------------------------------------------------------ heatmap head
// HeatmapHead.final_layer: 1x1 conv 32 -> K (17) + bias, f32 NCHW heatmaps out (the
// decode / moments input layout).  One lane per pixel: its 32 bf16 inputs (4 x 16 B),
// K x 32 f32 FMAs against weights that are uniform across the wave (scalar loads),
// K coalesced f32 plane stores.  Memory-bound (64 B in, 68 B out per pixel); the
// generic MFMA kernel spent 197 us per 1024 crops on it (masked 4x48 tiles, f32
// NCHW scatter).  Sums in f32 in channel order.
template <int KOUT>
__global__ __launch_bounds__(256) void head1x1_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      const float* __restrict__ bias, float* __restrict__ y,
                                                      long n_pix, int hw) {
    const long pix = (long)blockIdx.x * 256 + threadIdx.x;
    if (pix >= n_pix) return;
    float xv[32];
    const uint4* src = reinterpret_cast<const uint4*>(x + pix * 32);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 u = src[q];
        const uint32_t e[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            xv[q * 8 + 2 * j] = bf16_to_f32(e[j] & 0xffff);
            xv[q * 8 + 2 * j + 1] = bf16_to_f32(e[j] >> 16);
        }
    }
    const long n = pix / hw, pp = pix - n * hw;
    float* out = y + n * KOUT * hw + pp;
#pragma unroll
    for (int k = 0; k < KOUT; k++) {
        float acc = bias[k];
        const uint32_t* wk = reinterpret_cast<const uint32_t*>(w + k * 32);
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const uint32_t wp = wk[c];
            acc = __builtin_fmaf(bf16_to_f32(wp & 0xffff), xv[2 * c], acc);
            acc = __builtin_fmaf(bf16_to_f32(wp >> 16), xv[2 * c + 1], acc);
        }
        out[(long)k * hw] = acc;
    }
}

// Heatmap head with the last HRModule fuse folded in (graph pass head_fuse): the head's
// 32-ch input is out0 = act(sum_k nearest_up(in[k], 2^lg[k])) of the last stage's fuse
// layer; here each lane forms its pixel's out0 exactly as fuse_sum_kernel does (f32 sums
// in input order, ReLU, bf16 rounding) and feeds those values to head1x1_kernel's FMAs —
// bit-identical to the two launches, without writing / re-reading out0 (201 MB per 1024
// crops).  One grid row per crop.
struct HeadFuse {
    const uint16_t* in[4];
    int lg[4];
    int n_in, relu;
    const uint16_t* w;
    const float* bias;
    float* y;
    int H, W;
};

template <int KOUT>
__global__ __launch_bounds__(256) void head_fuse_kernel(HeadFuse p) {
    const int hw = p.H * p.W;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    if (i >= hw) return;
    const int yy = (int)((unsigned)i / (unsigned)p.W), xx = i - yy * p.W;
    float xv[32];
#pragma unroll
    for (int c = 0; c < 32; c++) xv[c] = 0.f;
    for (int k = 0; k < p.n_in; k++) {
        const int lg = p.lg[k];
        const int hs = p.H >> lg, ws = p.W >> lg;
        const uint4* src =
            reinterpret_cast<const uint4*>(p.in[k] + ((long)n * hs * ws + (yy >> lg) * ws + (xx >> lg)) * 32);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 u = src[q];
            const uint32_t e[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                xv[q * 8 + 2 * j] += bf16_to_f32(e[j] & 0xffff);
                xv[q * 8 + 2 * j + 1] += bf16_to_f32(e[j] >> 16);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 32; c++) {
        const float v = p.relu ? fmaxf(xv[c], 0.f) : xv[c];
        xv[c] = bf16_to_f32(f32_to_bf16(v));  // out0 as the fuse stores it
    }
    float* out = p.y + (long)n * KOUT * hw + i;
#pragma unroll
    for (int k = 0; k < KOUT; k++) {
        float acc = p.bias[k];
        const uint32_t* wk = reinterpret_cast<const uint32_t*>(p.w + k * 32);
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const uint32_t wp = wk[c];
            acc = __builtin_fmaf(bf16_to_f32(wp & 0xffff), xv[2 * c], acc);
            acc = __builtin_fmaf(bf16_to_f32(wp >> 16), xv[2 * c + 1], acc);
        }
        out[(long)k * hw] = acc;
    }
}

int g_cus1 = 0;

template <int BM, int KCH>
void launch_1x1(const P1x1& p, int cout_pad, hipStream_t s) {
    constexpr int lds = KCH * 4 * BM * 16;
    auto kern = conv1x1_kernel<BM, KCH>;
    static int per_cu = 0;
    if (per_cu == 0) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        MVP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds));
        if (per_cu < 1) per_cu = 1;
    }
    if (g_cus1 == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_cus1, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int y_blocks = cout_pad / BM;
    const long units = (p.n_pix + 16 * kPTW - 1) / (16 * kPTW);
    long gx = ((long)g_cus1 * per_cu + y_blocks - 1) / y_blocks;
    gx = std::min(gx, (units + 3) / 4);
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, (unsigned)y_blocks), dim3(256), lds, s, p);
    MVP_HIP(hipGetLastError());
}

template <int BM>
bool dispatch_k(const P1x1& p, int kch, int cout_pad, hipStream_t s) {
    switch (kch) {
        case 1: launch_1x1<BM, 1>(p, cout_pad, s); return true;
        case 2: launch_1x1<BM, 2>(p, cout_pad, s); return true;
        case 4: launch_1x1<BM, 4>(p, cout_pad, s); return true;
        case 8: launch_1x1<BM, 8>(p, cout_pad, s); return true;
        default: return false;
    }
}

}  // namespace

bool conv1x1_pair_supported(int cin_total, int cmid, int cout2) {
    const char* e = getenv("MVPOSE_NO_PAIRFUSE");  // diagnostics/tests: keep the two launches
    if (e && e[0] == '1') return false;
    return (cin_total == 64 || cin_total == 128) && cmid == 256 && cout2 == 64;
}

void launch_conv1x1_pair(const PairLaunch& c, hipStream_t s) {
    const int cin = c.c1 + (c.x2 ? c.c2 : 0);
    MVP_REQUIRE(conv1x1_pair_supported(cin, 256, 64), "conv1x1_pair: unsupported cin %d", cin);
    MVP_REQUIRE(c.c1 % 32 == 0 && c.c1 > 0 && (!c.x2 || c.c2 % 32 == 0), "conv1x1_pair: channel split %d/%d", c.c1,
                c.c2);
    if (c.n_pix == 0) return;
    PPair p{c.x, c.x2, c.c1, c.x2 ? c.c2 : 0, c.c1 / 32, c.w1, c.b1, c.res, c.y, c.w2, c.b2, c.y2,
            conv_zero_region(), c.n_pix};
    if (g_cus1 == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_cus1, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long units = (c.n_pix + 15) / 16;
    auto go = [&](auto kern, int kch) {
        const int kPairThreads = kch == 2 ? pair_threads<2>() : pair_threads<4>();
        const int lds = (kch * 4 * 256 + 8 * 4 * 64) * 16 + (kPairThreads / 64) * 4096;
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        int pc = 0;
        MVP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, kPairThreads, lds));
        if (pc < 1) pc = 1;
        const long grid = std::min<long>((long)g_cus1 * pc, (units + kPairThreads / 64 - 1) / (kPairThreads / 64));
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kPairThreads), lds, s, p);
    };
    // look-ahead depth (units in flight per wave) as measured best per join: 64-ch 1 (1,496 vs
    // 1,575 us per join graph with 2), the cat-fused 128-ch join 3
    MVP_REQUIRE(c.res || c.x2, "conv1x1_pair: a join without residual must be cat-fused");
    if (cin == 64) {
        MVP_REQUIRE(c.res != nullptr, "conv1x1_pair: 64-ch join needs its residual");
        go(conv1x1_pair_kernel<2, true, 1>, 2);
    } else if (c.res) {
        go(conv1x1_pair_kernel<4, true, 1>, 4);
    } else {
        go(conv1x1_pair_kernel<4, false, 3>, 4);
    }
    MVP_HIP(hipGetLastError());
}

// A 1x1 conv 64 -> 256 (or the cat-fused 64 + 64 -> 256) with ReLU, + optional 256-ch
// residual, on the Bottleneck-join kernel without its second GEMM: one wave owns all 256
// couts of 16 pixels (input read once instead of once per 128-cout column block) and its
// residual loads / output stores go through LDS as whole 256-B runs.
bool launch_conv1x1_wide(const ConvLaunch& c, hipStream_t s) {
    const int cin = c.Cin;
    if (c.ks != 1 || c.stride != 1 || c.out_f32_nchw || c.Cout != 256 || !c.relu) return false;
    if (!(cin == 64 || (cin == 128 && c.x2 && c.c1 == 64))) return false;
    if (cin == 64 && !c.res) return false;
    const long n_pix = (long)c.N * c.H * c.W;
    if (n_pix == 0) return true;
    PPair p{c.x, c.x2, 64, cin == 128 ? 64 : 0, 2, c.w, c.bias, c.res, c.y, nullptr, nullptr,
            nullptr, conv_zero_region(), n_pix};
    if (g_cus1 == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_cus1, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long units = (n_pix + 15) / 16;
    auto go = [&](auto kern, int kch) {
        const int lds = kch * 4 * 256 * 16 + 8 * 4096;
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        int pc = 0;
        MVP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, 512, lds));
        if (pc < 1) pc = 1;
        const long grid = std::min<long>((long)g_cus1 * pc, (units + 7) / 8);
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, s, p);
    };
    if (cin == 64) go(conv1x1_pair_kernel<2, true, 1, false>, 2);
    else if (c.res) go(conv1x1_pair_kernel<4, true, 1, false>, 4);
    else go(conv1x1_pair_kernel<4, false, 1, false>, 4);
    MVP_HIP(hipGetLastError());
    return true;
}

bool launch_head1x1(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 1 || c.stride != 1 || !c.out_f32_nchw || c.Cin != 32 || c.Cout != 17 || c.res || c.relu || c.x2)
        return false;
    const char* e = getenv("MVPOSE_NO_HEAD1X1");  // diagnostics/tests: generic conv kernel
    if (e && e[0] == '1') return false;
    const long n_pix = (long)c.N * c.H * c.W;
    if (n_pix == 0) return true;
    hipLaunchKernelGGL(head1x1_kernel<17>, dim3((unsigned)((n_pix + 255) / 256)), dim3(256), 0, s, c.x, c.w, c.bias,
                       c.yf, n_pix, c.H * c.W);
    MVP_HIP(hipGetLastError());
    return true;
}

bool head_fuse_supported(int cin, int cout, int n_in) {
    const char* e = getenv("MVPOSE_NO_HEADFUSE");  // diagnostics/tests: fuse_sum + head1x1
    if (e && e[0] == '1') return false;
    const char* e2 = getenv("MVPOSE_NO_HEAD1X1");
    if (e2 && e2[0] == '1') return false;
    return cin == 32 && cout == 17 && n_in >= 1 && n_in <= 4;
}

void launch_head_fuse(const uint16_t* const* in, const int* up, int n_in, int relu, const uint16_t* w,
                      const float* bias, float* y, int N, int H, int W, hipStream_t s) {
    MVP_REQUIRE(n_in >= 1 && n_in <= 4, "head_fuse: n_in=%d", n_in);
    HeadFuse p{};
    for (int k = 0; k < n_in; k++) {
        int lg = 0;
        while ((1 << lg) < up[k]) lg++;
        MVP_REQUIRE(up[k] == (1 << lg) && H % up[k] == 0 && W % up[k] == 0, "head_fuse: upsample factor %d", up[k]);
        p.in[k] = in[k];
        p.lg[k] = lg;
    }
    p.n_in = n_in;
    p.relu = relu;
    p.w = w;
    p.bias = bias;
    p.y = y;
    p.H = H;
    p.W = W;
    MVP_REQUIRE((long)H * W < (1L << 30) && N < 65536, "head_fuse: sizes");
    if (N == 0) return;
    hipLaunchKernelGGL(head_fuse_kernel<17>, dim3((unsigned)((H * W + 255) / 256), (unsigned)N), dim3(256), 0, s, p);
    MVP_HIP(hipGetLastError());
}

bool launch_conv1x1_direct(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 1 || c.stride != 1 || c.out_f32_nchw || c.Cin % 32 != 0) return false;
    if (launch_conv1x1_wide(c, s)) return true;
    const int bm = conv_cout_pad(c.Cout) % 128 == 0 && c.Cin <= 64 ? 128 : conv_cout_pad(c.Cout) % 64 == 0 ? 64 : 32;
    if (c.Cout % (bm / 4) != 0) return false;  // lane groups own bm/4 consecutive couts
    const int cout_pad = conv_cout_pad(c.Cout);
    const int kch = c.Cin / 32;
    P1x1 p{c.x, c.w, c.bias, c.res, c.y, conv_zero_region(), (long)c.N * c.H * c.W, c.Cout, c.relu,
           nullptr, c.Cin, 0, c.Cin / 32};
    if (c.x2) {  // dual input: c.Cin = c1 + c2
        MVP_REQUIRE(c.c1 % 32 == 0 && c.c1 > 0 && c.c1 < c.Cin, "conv1x1: dual input split %d of %d", c.c1, c.Cin);
        p.x2 = c.x2;
        p.c1 = c.c1;
        p.c2 = c.Cin - c.c1;
        p.kch1 = c.c1 / 32;
    }
    if (p.n_pix == 0) return true;
    if (cout_pad % 128 == 0 && kch <= 2) {  // 128 couts: registers allow K <= 64
        if (kch == 1) launch_1x1<128, 1>(p, cout_pad, s);
        else launch_1x1<128, 2>(p, cout_pad, s);
        return true;
    }
    if (cout_pad % 64 == 0) return dispatch_k<64>(p, kch, cout_pad, s);
    return dispatch_k<32>(p, kch, cout_pad, s);
}

}  // namespace mvp
