// HRNet-W32 convolutions for gfx950: implicit GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16).
//
// GEMM view per conv:  Y[cout][pix] = sum_k W[cout][k] * X[k][pix],  k = (kh, kw, cin),
// activations NHWC bf16 so 8 consecutive k of one tap are 16 contiguous bytes.
// A = weights (rows = couts), B = im2col activations (cols = output pixels); the
// accumulator lane layout (col = lane&15 -> pixel, rows (lane>>4)*4+r -> 4
// consecutive couts) gives an 8-byte NHWC store per lane.
//
// Each 256-thread workgroup (4 waves) owns an output tile of NB crops x TH x TW
// pixels x BM couts.  Per 32-channel input chunk it stages the input HALO of the
// tile ((TH-1)*S+KS) x ((TW-1)*S+KS) and the BM x KS*KS x 32 weight slice in LDS,
// so every input pixel is fetched from L2/HBM once per tile instead of KS*KS times
// (im2col happens in the LDS addressing).  Rows are padded by 16 B to break the
// 64-B-stride bank pattern of the ds_read_b128 fragment reads.  Epilogue fuses
// folded-BN bias, optional residual add (BasicBlock/Bottleneck), ReLU and bf16
// pack; the head variant writes f32 NCHW heatmaps.
#include "conv.h"

#include <cstdlib>
#include <type_traits>
#include "mvp_common.h"

namespace mvp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN preserved
    return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float silu(float v) { return v * __builtin_amdgcn_rcpf(1.f + __expf(-v)); }

struct ConvParams {
    const uint16_t* __restrict__ x;
    const uint16_t* __restrict__ w;
    const float* __restrict__ bias;
    const uint16_t* __restrict__ res;
    uint16_t* __restrict__ y;
    float* __restrict__ yf;
    const uint16_t* __restrict__ zero;  // kZeroSlots*16 zero bytes: source of padding / out-of-image slots
    uint16_t* sink;                     // write-only scratch for masked-off lanes' stores
    float* sinkf;
    int N, H, W, Cin, Ho, Wo, Cout, Cout_pad;
    int xs, ys, rs;  // pixel strides (elements) of x / y / res
    int relu, out_f32;  // relu: 0 none, 1 ReLU, 2 SiLU
    int tiles_w, tiles_h, n_tiles;
    int wmode;  // WM_ONCE / WM_RESIDENT / WM_STREAM
};

constexpr int kZeroSlots = 4096;  // 16-B slots of the zero region (64 KiB)

// Weight staging modes: one 32-channel chunk staged once (Cin = 32); every chunk
// resident in LDS for the whole launch (fits); or a per-chunk double buffer.
enum { WM_ONCE = 0, WM_RESIDENT = 1, WM_STREAM = 2 };

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

template <int KS, int S, int BM, int TH, int TW, int NB, int NW = 4>
struct ConvCfg {
    static constexpr int HH = (TH - 1) * S + KS;
    static constexpr int HW = (TW - 1) * S + KS;
    static constexpr int KK = KS * KS;
    static constexpr int HALO_PIX = NB * HH * HW;
    static constexpr int HGRAN = 16 * NW;  // whole 1-KiB DMA pieces for every wave in each round
    static constexpr int HPIX = (HALO_PIX + HGRAN - 1) / HGRAN * HGRAN;  // pixels per chunk plane
    static constexpr int H_SLOTS = 4 * HPIX;                // 16-B slots, layout [chunk q][pixel]
    static constexpr int W_SLOTS = KK * 4 * BM;             // layout [tap][chunk q][cout]
    static constexpr int H_BYTES = H_SLOTS * 16;
    static constexpr int W_BYTES = (W_SLOTS + 63) / 64 * 1024;
    static int lds_bytes(int wmode, int n_chunks, int nbuf) {
        return nbuf * H_BYTES + (wmode == WM_ONCE ? 1 : wmode == WM_RESIDENT ? n_chunks : nbuf) * W_BYTES;
    }
};

// s_waitcnt vmcnt(n') for the largest level n' <= n: waits until at most n' of this
// wave's vector-memory operations are outstanding (rounding down only waits longer).
__device__ __forceinline__ void wait_vmcnt_le(int n) {
    if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Persistent implicit-GEMM conv with an NBUF-deep LDS-DMA ring.  A workgroup walks
// its work items k = (tile, 32-channel chunk); the halo (+ weight slice when
// streamed) of item k+NBUF-1 is issued by global_load_lds straight into the ring
// slot freed by item k-1, so NBUF-1 items' DMAs are in flight under each item's
// MFMAs.  Completion is tracked per wave by counting its own vector-memory
// instructions (DMA pieces, residual loads, stores — every one issued
// unconditionally, out-of-range lanes pointed at a zero region / a sink), so the
// top-of-item wait is vmcnt(#ops younger than item k's DMA), never vmcnt(0).
// LDS images are chunk-major ([q][pixel] halo, [tap][q][cout] weights): each
// 16-lane ds_read_b128 group of a fragment read touches 16 distinct bank slots.
template <int KS, int S, int BM, int TH, int TW, int NB, int NBUF, int NW>
__global__ __launch_bounds__(NW * 64, 2) void conv_mfma_kernel(ConvParams p) {
    using C = ConvCfg<KS, S, BM, TH, TW, NB, NW>;
    constexpr int NT = NW * 64;  // threads
    constexpr int PAD = KS / 2;
    constexpr int HH = C::HH, HW = C::HW, KK = C::KK, HPIX = C::HPIX;
    constexpr int P = NB * TH * TW;
    static_assert(P % 64 == 0, "tile must hold a multiple of 64 pixels");
    static_assert(NBUF >= 2, "ring needs two slots");
    constexpr int D = NBUF - 1;  // items in flight ahead of the one computing
    constexpr int NPT = P / 16;
    constexpr int NCT = BM / 16;
    static_assert(NPT % NW == 0, "pixel tiles must split evenly over the waves");
    constexpr int PTW = NPT / NW;  // pixel tiles per wave
    static_assert(C::H_SLOTS % NT == 0, "halo pieces must split evenly over the waves");
    constexpr int kHaloOps = C::H_SLOTS / NT;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    const int co0 = blockIdx.y * BM;
    const int n_chunks = p.Cin >> 5;
    const int wmode = p.wmode;
    const size_t plane_in = (size_t)p.H * p.W;
    const int w_ops = (C::W_SLOTS - wave * 64 + NT - 1) / NT;  // weight-slice DMA pieces issued by this wave
    const int item_ops = kHaloOps + (wmode == WM_STREAM ? w_ops : 0);
    const int n_items = ((p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) * n_chunks;
    auto halo_buf = [&](int b) -> uint8_t* { return lds + b * C::H_BYTES; };
    auto w_buf = [&](int b, int chunk) -> uint8_t* {
        const int slot = wmode == WM_ONCE ? 0 : wmode == WM_RESIDENT ? chunk : b;
        return lds + NBUF * C::H_BYTES + slot * C::W_BYTES;
    };

    // B fragment: lane reads pixel (lane & 15) of its pixel tile, chunk q = lane >> 4
    int hbase[PTW];
#pragma unroll
    for (int i = 0; i < PTW; i++) {
        const int pp = (wave * PTW + i) * 16 + (lane & 15);
        const int nb = pp / (TH * TW);
        const int r = pp - nb * (TH * TW);
        const int th = r / TW, tw = r - (r / TW) * TW;
        hbase[i] = ((lane >> 4) * HPIX + (nb * HH + th * S) * HW + tw * S) * 8;
    }
    const int abase = ((lane >> 4) * BM + (lane & 15)) * 8;
    // folded-BN bias of this block's couts, read by the epilogue from LDS (visible after
    // the first item's barrier); registers would pin a pending load across the loop
    __shared__ float4 sbias[BM / 4];
    if (tid < BM / 4) sbias[tid] = *reinterpret_cast<const float4*>(p.bias + co0 + tid * 4);

    auto tile_origin = [&](int tile, int& n0, int& ho0, int& wo0) {
        const int tw_i = tile % p.tiles_w;
        const int t2 = tile / p.tiles_w;
        n0 = (t2 / p.tiles_h) * NB;
        ho0 = (t2 % p.tiles_h) * TH;
        wo0 = tw_i * TW;
    };
    auto issue_w = [&](int chunk, uint8_t* wb) {
        const uint16_t* wsrc = p.w + (size_t)co0 * KK * p.Cin + chunk * 32;
#pragma unroll
        for (int s0 = 0; s0 < C::W_SLOTS; s0 += NT) {
            const int sw0 = s0 + wave * 64;
            if (sw0 < C::W_SLOTS) {  // wave-uniform: exactly w_ops pieces per call
                const int sl = sw0 + lane;
                const void* src = p.zero + (sl & (kZeroSlots - 1)) * 8;
                if (sl < C::W_SLOTS) {
                    const int co = sl % BM, tq = sl / BM;  // tq = tap * 4 + q
                    src = wsrc + ((size_t)co * KK + (tq >> 2)) * p.Cin + (tq & 3) * 8;
                }
                glds16(src, wb + sw0 * 16);
            }
        }
    };
    // Per-lane halo geometry of each of this wave's DMA pieces, fixed for the launch:
    // pixel (nb, hh, ww) of the halo and its element offset from the halo origin.
    // Per item only the tile origin moves: bounds = 3 compares, address = one add.
    int hgeo[kHaloOps], hoff[kHaloOps];
#pragma unroll
    for (int j = 0; j < kHaloOps; j++) {
        const int sw0 = j * NT + wave * 64;
        const int q = sw0 / HPIX;
        const int pix = sw0 - q * HPIX + lane;
        const int nb = pix / (HH * HW);
        const int r = pix - nb * (HH * HW);
        const int hh = r / HW, ww = r - (r / HW) * HW;
        hgeo[j] = pix < C::HALO_PIX ? (hh | (ww << 10) | (nb << 20)) : -1;
        hoff[j] = (int)(((size_t)nb * plane_in + (size_t)hh * p.W + ww) * p.xs) + q * 8;
    }
    auto issue = [&](int k, int buf) {
        const int tile = blockIdx.x + (k / n_chunks) * gridDim.x, chunk = k % n_chunks;
        int n0, ho0, wo0;
        tile_origin(tile, n0, ho0, wo0);
        const int hi0 = ho0 * S - PAD, wi0 = wo0 * S - PAD;
        // element offset of the halo origin (may point before the image; only in-bounds lanes use it)
        const uint16_t* xb = p.x + ((long)n0 * (long)plane_in + (long)hi0 * p.W + wi0) * p.xs + chunk * 32;
        uint8_t* hb = halo_buf(buf);
#pragma unroll
        for (int j = 0; j < kHaloOps; j++) {
            const int sw0 = j * NT + wave * 64;  // this wave's 64-slot piece (one chunk plane)
            const int g = hgeo[j];
            const int hh = g & 1023, ww = (g >> 10) & 1023, nb = g >> 20;
            const bool in = g >= 0 && (unsigned)(hi0 + hh) < (unsigned)p.H && (unsigned)(wi0 + ww) < (unsigned)p.W &&
                            n0 + nb < p.N;
            // out-of-image slots read zeros from a 64-KiB zero region, one distinct 16-B
            // slot per lane: a single shared zero line is an L2-channel hot spot
            const void* src = in ? (const void*)(xb + hoff[j]) : (const void*)(p.zero + ((sw0 + lane) & (kZeroSlots - 1)) * 8);
            glds16(src, hb + sw0 * 16);
        }
        if (wmode == WM_STREAM) issue_w(chunk, w_buf(buf, chunk));
    };
    // Per-lane output pixel of each pixel tile relative to the tile origin.
    int eoff[PTW], egeo[PTW];
#pragma unroll
    for (int i = 0; i < PTW; i++) {
        const int pp = (wave * PTW + i) * 16 + (lane & 15);
        const int nb = pp / (TH * TW);
        const int r = pp - nb * (TH * TW);
        const int th = r / TW, tw = r - (r / TW) * TW;
        egeo[i] = th | (tw << 10) | (nb << 20);
        eoff[i] = (nb * p.Ho + th) * p.Wo + tw;
    }
    f32x4 acc[PTW][NCT];
#pragma unroll
    for (int i = 0; i < PTW; i++)
#pragma unroll
        for (int c = 0; c < NCT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- prologue: resident / single weight slices, then the first D items
    int ops = 0;
    if (wmode == WM_ONCE) {
        issue_w(0, w_buf(0, 0));
        ops += w_ops;
    } else if (wmode == WM_RESIDENT) {
        for (int c = 0; c < n_chunks; c++) issue_w(c, w_buf(0, c));
        ops += w_ops * n_chunks;
    }
    int mark[D];  // ops count at the end of item (k + j)'s DMA, j = 0 .. D-1
#pragma unroll
    for (int j = 0; j < D; j++) {
        if (j < n_items) {
            issue(j, j);
            ops += item_ops;
        }
        mark[j] = ops;
    }

    const int store_ops = p.out_f32 ? 4 * PTW * NCT : PTW * NCT;
    int buf = 0;
    for (int k = 0; k < n_items; k++) {
        // item k's pieces from this wave have landed; the barrier makes every wave's
        // pieces visible and guarantees all waves are done reading ring slot k-1
        wait_vmcnt_le(ops - mark[0]);
        // plain s_barrier, not __syncthreads(): its release fence would drain vmcnt to 0
        // (every DMA in flight, stores included) and collapse the ring to depth 1
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j + 1 < D; j++) mark[j] = mark[j + 1];
        const int tile = blockIdx.x + (k / n_chunks) * gridDim.x, chunk = k % n_chunks;
        int n0, ho0, wo0;
        tile_origin(tile, n0, ho0, wo0);
        const int pix0 = (n0 * p.Ho + ho0) * p.Wo + wo0;  // output pixel of the tile origin
        const int co_l = co0 + (lane >> 4) * 4;
        // One body per item kind, so residual loads and their use sit on the same
        // control path (the waitcnt pass merges paths, and a load pending on an
        // infeasible path would cost a vmcnt(0) at the next item).
        auto item = [&](auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        // residual rows of this tile (before the next DMA so they land under the MFMAs);
        // issued for every last-chunk item, from the zero region when there is no residual
        uint2 resv[PTW][NCT];
        if constexpr (LAST) {
#pragma unroll
            for (int i = 0; i < PTW; i++) {
                const int g = egeo[i];
                const bool valid = n0 + (g >> 20) < p.N && ho0 + (g & 1023) < p.Ho && wo0 + ((g >> 10) & 1023) < p.Wo;
                const uint16_t* rrow = (p.res ? p.res : p.zero) + (size_t)(pix0 + eoff[i]) * p.rs;
#pragma unroll
                for (int c = 0; c < NCT; c++) {
                    const int co = co_l + c * 16;
                    const uint16_t* src = (p.res && valid && co < p.Cout) ? rrow + co : p.zero + lane * 4;
                    resv[i][c] = *reinterpret_cast<const uint2*>(src);
                }
            }
            ops += PTW * NCT;
        }
        asm volatile("" ::: "memory");
        // issued for every item (past the end: a tile beyond the last crop, i.e. zero-region
        // reads into the free slot), so the VMEM count between the residual loads and their
        // use is the same on every path and the epilogue waits vmcnt(pieces), not vmcnt(0)
        const int nbuf = buf + D >= NBUF ? buf + D - NBUF : buf + D;
        issue(k + D, nbuf);
        ops += item_ops;
        mark[D - 1] = ops;
        asm volatile("" ::: "memory");
        const uint16_t* sh = reinterpret_cast<const uint16_t*>(halo_buf(buf));
        const uint16_t* sw = reinterpret_cast<const uint16_t*>(w_buf(buf, chunk));
        // fragment reads of tap t+1 are issued before the MFMAs of tap t (two static
        // register sets), so LDS latency hides under the matrix work
        bf16x8 fa[2][NCT], fb[2][PTW];
        auto load_tap = [&](int tap, bf16x8 (&a)[NCT], bf16x8 (&b)[PTW]) {
            const int toff = ((tap / KS) * HW + (tap % KS)) * 8;
#pragma unroll
            for (int c = 0; c < NCT; c++)
                a[c] = *reinterpret_cast<const bf16x8*>(sw + tap * 4 * BM * 8 + abase + c * 16 * 8);
#pragma unroll
            for (int i = 0; i < PTW; i++) b[i] = *reinterpret_cast<const bf16x8*>(sh + hbase[i] + toff);
        };
        load_tap(0, fa[0], fb[0]);
#pragma unroll
        for (int tap = 0; tap < KK; tap++) {
            const int cur = tap & 1;
            if (tap + 1 < KK) load_tap(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);  // keep tap t+1's reads ahead of tap t's MFMAs
#pragma unroll
            for (int i = 0; i < PTW; i++)
#pragma unroll
                for (int c = 0; c < NCT; c++)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][c], fb[cur][i], acc[i][c], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (LAST) {
            // ---- epilogue: + bias [+ residual] [relu] -> bf16 NHWC (or f32 NCHW for the head);
            // every store instruction issues (invalid lanes write the sink)
#pragma unroll
            for (int i = 0; i < PTW; i++) {
                const int g = egeo[i];
                const int nb = g >> 20, th = g & 1023, tw = (g >> 10) & 1023;
                const int n = n0 + nb, ho = ho0 + th, wo = wo0 + tw;
                const bool valid = n < p.N && ho < p.Ho && wo < p.Wo;
                const int pix = pix0 + eoff[i];
                uint16_t* yrow = p.y + (size_t)pix * p.ys;
#pragma unroll
                for (int c = 0; c < NCT; c++) {
                    const int co = co_l + c * 16;
                    const float4 bias = sbias[c * 4 + (lane >> 4)];
                    float v0 = acc[i][c][0] + bias.x, v1 = acc[i][c][1] + bias.y;
                    float v2 = acc[i][c][2] + bias.z, v3 = acc[i][c][3] + bias.w;
                    acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (p.out_f32) {
                        const size_t plane = (size_t)p.Ho * p.Wo;
                        const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const bool ok = valid && co + q < p.Cout;
                            float* dst = ok ? p.yf + ((size_t)n * p.Cout + co + q) * plane + (size_t)ho * p.Wo + wo
                                            : p.sinkf + lane * 4 + q;
                            *dst = vv[q];
                        }
                        continue;
                    }
                    if (p.relu == 2) {  // SiLU, then the residual (CSPNeXtBlock: conv2(conv1(x)) + x)
                        v0 = silu(v0);
                        v1 = silu(v1);
                        v2 = silu(v2);
                        v3 = silu(v3);
                    }
                    {  // + residual (zeros when the conv has none)
                        const uint2 rv = resv[i][c];
                        v0 += bf16_to_f32(rv.x & 0xffff);
                        v1 += bf16_to_f32(rv.x >> 16);
                        v2 += bf16_to_f32(rv.y & 0xffff);
                        v3 += bf16_to_f32(rv.y >> 16);
                    }
                    if (p.relu == 1) {  // ReLU after the residual (HRNet BasicBlock / Bottleneck)
                        v0 = fmaxf(v0, 0.f);
                        v1 = fmaxf(v1, 0.f);
                        v2 = fmaxf(v2, 0.f);
                        v3 = fmaxf(v3, 0.f);
                    }
                    uint2 o;
                    o.x = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                    o.y = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
                    uint16_t* dst = (valid && co < p.Cout) ? yrow + co : p.sink + lane * 4;
                    *reinterpret_cast<uint2*>(dst) = o;
                }
            }
            ops += store_ops;
        }
        };
        if (chunk == n_chunks - 1)
            item(std::integral_constant<bool, true>{});
        else
            item(std::integral_constant<bool, false>{});
        buf = buf + 1 == NBUF ? 0 : buf + 1;
    }
}

int g_num_cus = 0;
uint16_t* g_zero = nullptr;

int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    return g_num_cus;
}

uint16_t* g_sink = nullptr;

const uint16_t* zero_page() {
    if (!g_zero) {
        MVP_HIP(hipMalloc(&g_zero, kZeroSlots * 16));
        MVP_HIP(hipMemset(g_zero, 0, kZeroSlots * 16));
        MVP_HIP(hipMalloc(&g_sink, 64 * 16));
    }
    return g_zero;
}

constexpr int kLdsMax = 160 * 1024 - 1024;  // dynamic LDS budget (static: the bias tile)

// Resident workgroups per CU of one kernel instance at a given LDS footprint (cached).
template <int KS, int S, int BM, int TH, int TW, int NB, int NBUF, int NW>
int blocks_per_cu(int lds) {
    auto kern = conv_mfma_kernel<KS, S, BM, TH, TW, NB, NBUF, NW>;
    static bool attr_set = false;
    if (!attr_set) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
        attr_set = true;
    }
    static int cache[kLdsMax / 1024 + 1] = {0};
    int& per_cu = cache[(lds + 1023) / 1024];
    if (per_cu == 0) {
        MVP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NW * 64, lds));
        if (per_cu < 1) per_cu = 1;
    }
    return per_cu;
}

template <int KS, int S, int BM, int TH, int TW, int NB, int NBUF, int NW>
void launch_ring(const ConvParams& p, int lds, int per_cu, hipStream_t s) {
    const int y_blocks = p.Cout_pad / BM;
    long gx = ((long)num_cus() * per_cu + y_blocks - 1) / y_blocks;
    if (gx > p.n_tiles) gx = p.n_tiles;
    hipLaunchKernelGGL((conv_mfma_kernel<KS, S, BM, TH, TW, NB, NBUF, NW>), dim3((unsigned)gx, (unsigned)y_blocks),
                       dim3(NW * 64), lds, s, p);
}

template <int KS, int S, int BM, int TH, int TW, int NB, int NW>
int wmode_for(int n_chunks) {
    using C = ConvCfg<KS, S, BM, TH, TW, NB, NW>;
    return n_chunks == 1 ? WM_ONCE : C::lds_bytes(WM_RESIDENT, n_chunks, 2) <= kLdsMax ? WM_RESIDENT : WM_STREAM;
}

// Resident workgroups per CU by LDS alone for the 2-slot ring (tile / wave-count choice).
template <int KS, int S, int BM, int TH, int TW, int NB, int NW>
int lds_blocks(int n_chunks) {
    using C = ConvCfg<KS, S, BM, TH, TW, NB, NW>;
    return kLdsMax / C::lds_bytes(wmode_for<KS, S, BM, TH, TW, NB, NW>(n_chunks), n_chunks, 2);
}

template <int KS, int S, int BM, int TH, int TW, int NB, int NW>
void launch_cfg(const ConvParams& p0, hipStream_t s) {
    using C = ConvCfg<KS, S, BM, TH, TW, NB, NW>;
    ConvParams p = p0;
    p.tiles_w = (p.Wo + TW - 1) / TW;
    p.tiles_h = (p.Ho + TH - 1) / TH;
    const long tiles_n = (p.N + NB - 1) / NB;
    const long nt = tiles_n * p.tiles_h * p.tiles_w;
    MVP_REQUIRE(nt < (1L << 31), "conv: too many tiles");
    p.n_tiles = (int)nt;
    p.zero = zero_page();
    p.sink = g_sink;
    p.sinkf = reinterpret_cast<float*>(g_sink);
    const int n_chunks = p.Cin / 32;
    p.wmode = wmode_for<KS, S, BM, TH, TW, NB, NW>(n_chunks);
    // ring depth: maximise DMA items in flight per CU = resident workgroups x (depth - 1)
    int best = 0, best_score = -1, best_lds = 0, best_bpc = 0;
    for (int nbuf = 2; nbuf <= 4; nbuf++) {
        const int lds = C::lds_bytes(p.wmode, n_chunks, nbuf);
        if (lds > kLdsMax) break;
        const int bpc = nbuf == 2   ? blocks_per_cu<KS, S, BM, TH, TW, NB, 2, NW>(lds)
                        : nbuf == 3 ? blocks_per_cu<KS, S, BM, TH, TW, NB, 3, NW>(lds)
                                    : blocks_per_cu<KS, S, BM, TH, TW, NB, 4, NW>(lds);
        const int score = bpc * (nbuf - 1);
        if (score > best_score) {
            best = nbuf;
            best_score = score;
            best_lds = lds;
            best_bpc = bpc;
        }
    }
    MVP_REQUIRE(best > 0, "conv: LDS %d B over budget", C::lds_bytes(p.wmode, n_chunks, 2));
    if (best == 2)
        launch_ring<KS, S, BM, TH, TW, NB, 2, NW>(p, best_lds, best_bpc, s);
    else if (best == 3)
        launch_ring<KS, S, BM, TH, TW, NB, 3, NW>(p, best_lds, best_bpc, s);
    else
        launch_ring<KS, S, BM, TH, TW, NB, 4, NW>(p, best_lds, best_bpc, s);
}

// Cout tile: 64 couts when the weights can stay LDS-resident (or Cin = 32),
// else 32 couts if that makes them resident, else 64 couts streamed per chunk.
template <int KS, int S, int TH, int TW, int NB, int NW>
void launch_tile(const ConvParams& p, hipStream_t s) {
    const int n_chunks = p.Cin / 32;
    if (p.Cout_pad == 32) return launch_cfg<KS, S, 32, TH, TW, NB, NW>(p, s);
    if (n_chunks == 1 || ConvCfg<KS, S, 64, TH, TW, NB, NW>::lds_bytes(WM_RESIDENT, n_chunks, 2) <= kLdsMax)
        return launch_cfg<KS, S, 64, TH, TW, NB, NW>(p, s);
    if (ConvCfg<KS, S, 32, TH, TW, NB, NW>::lds_bytes(WM_RESIDENT, n_chunks, 2) <= kLdsMax)
        return launch_cfg<KS, S, 32, TH, TW, NB, NW>(p, s);
    launch_cfg<KS, S, 64, TH, TW, NB, NW>(p, s);
}

// 4-wave tile (TH, TW, NB) unless its LDS footprint leaves one workgroup per CU
// (one wave per SIMD: nothing hides LDS / DMA / barrier latency behind another
// wave's MFMAs) — then the 8-wave tile (TH8, TW8, NB8), twice the pixels, one
// workgroup of two waves per SIMD sharing the resident weights.
template <int KS, int S, int TH, int TW, int NB, int TH8, int TW8, int NB8>
void launch_tile2(const ConvParams& p, hipStream_t s) {
    const int n_chunks = p.Cin / 32;
    const int bm = p.Cout_pad == 32                                                               ? 32
                   : (n_chunks == 1 || ConvCfg<KS, S, 64, TH, TW, NB>::lds_bytes(WM_RESIDENT, n_chunks, 2) <= kLdsMax)
                       ? 64
                   : ConvCfg<KS, S, 32, TH, TW, NB>::lds_bytes(WM_RESIDENT, n_chunks, 2) <= kLdsMax ? 32
                                                                                                    : 64;
    const int blocks4 = bm == 32 ? lds_blocks<KS, S, 32, TH, TW, NB, 4>(n_chunks)
                                 : lds_blocks<KS, S, 64, TH, TW, NB, 4>(n_chunks);
    const bool eight = blocks4 < 2;
    if (eight)
        launch_tile<KS, S, TH8, TW8, NB8, 8>(p, s);
    else
        launch_tile<KS, S, TH, TW, NB, 4>(p, s);
}

// Tile shape per output plane.
template <int KS, int S>
void launch_plane(const ConvParams& p, hipStream_t s) {
    if constexpr (S == 1) {
        if (p.Wo == 48 && p.Ho % 8 == 0)
            launch_tile2<KS, S, 4, 48, 1, 8, 48, 1>(p, s);
        else if (p.Wo == 24 && p.Ho % 16 == 0)
            launch_tile2<KS, S, 8, 24, 1, 16, 24, 1>(p, s);
        else if (p.Wo == 12 && p.Ho == 16)
            launch_tile2<KS, S, 16, 12, 1, 16, 12, 2>(p, s);
        else if (p.Wo == 6 && p.Ho == 8)
            launch_tile2<KS, S, 8, 6, 4, 8, 6, 8>(p, s);
        else
            launch_tile<KS, S, 4, 16, 1, 4>(p, s);  // generic masked tiling
    } else {
        const char* e = getenv("MVPOSE_S2_TILE");  // tuning experiments only
        const int v = e ? atoi(e) : 0;  // 7: the pre-sweep 4-wave default
        if (v == 1 && p.Wo % 8 == 0 && p.Ho % 16 == 0) return launch_tile<KS, S, 16, 8, 1, 4>(p, s);
        if (v == 2 && p.Wo % 8 == 0 && p.Ho % 8 == 0) return launch_tile<KS, S, 8, 8, 2, 4>(p, s);
        if (v == 3 && p.Wo % 16 == 0 && p.Ho % 8 == 0) return launch_tile<KS, S, 8, 16, 1, 4>(p, s);
        if (v == 4 && p.Wo % 16 == 0 && p.Ho % 4 == 0) return launch_tile<KS, S, 4, 16, 2, 4>(p, s);
        if (v == 5 && p.Wo % 8 == 0 && p.Ho % 16 == 0) return launch_tile<KS, S, 16, 8, 1, 8>(p, s);
        if (v == 6 && p.Wo % 16 == 0 && p.Ho % 8 == 0) return launch_tile<KS, S, 8, 16, 1, 8>(p, s);
        // Cin >= 64 (stem conv2 64@128x96, transition1.1 256@64x48): 16x8-pixel tiles on
        // 8 waves (2 per SIMD) sharing one weight slice — 800 -> 650-710 us and
        // 1052 -> 771 us per 1024 crops (tools/s2_tile_sweep.py); the 32-ch planes keep
        // the 4-wave tiles (55 vs 62 us)
        if (v == 0 && p.Cin >= 64 && p.Wo % 8 == 0 && p.Ho % 16 == 0)
            launch_tile<KS, S, 16, 8, 1, 8>(p, s);
        else if (p.Wo % 16 == 0 && p.Ho % 4 == 0)
            launch_tile<KS, S, 4, 16, 1, 4>(p, s);
        else if (p.Wo % 8 == 0 && p.Ho % 8 == 0)
            launch_tile<KS, S, 8, 8, 1, 4>(p, s);
        else if (p.Wo % 4 == 0 && p.Ho % 16 == 0)
            launch_tile<KS, S, 16, 4, 1, 4>(p, s);
        else
            launch_tile<KS, S, 4, 16, 1, 4>(p, s);
    }
}

// ---------------------------------------------------------------- stem conv
// 3x3/s2, 4 -> 64 channels, direct (VALU fp32): 0.3% of the network's MACs.
// One thread = one output pixel x 16 output channels (4 threads per pixel).
__global__ __launch_bounds__(256) void stem_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, uint16_t* __restrict__ y, int N,
                                                   int H, int W, int Ho, int Wo) {
    __shared__ float sw[36][64];
    __shared__ float sb[64];
    for (int i = threadIdx.x; i < 36 * 64; i += 256) {
        const int co = i / 36, k = i % 36;  // w layout [co][tap][c]
        sw[k][co] = w[i];
    }
    if (threadIdx.x < 64) sb[threadIdx.x] = bias[threadIdx.x];
    __syncthreads();
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const int grp = gid & 3;
    const long pix = gid >> 2;
    if (pix >= (long)N * Ho * Wo) return;
    const int wo = pix % Wo;
    const int ho = (pix / Wo) % Ho;
    const int n = pix / ((long)Wo * Ho);
    const int cb = grp * 16;
    float acc[16];
#pragma unroll
    for (int c = 0; c < 16; c++) acc[c] = sb[cb + c];
    for (int kh = 0; kh < 3; kh++) {
        const int hi = ho * 2 - 1 + kh;
        for (int kw = 0; kw < 3; kw++) {
            const int wi = wo * 2 - 1 + kw;
            float xin[3] = {0.f, 0.f, 0.f};
            if (hi >= 0 && hi < H && wi >= 0 && wi < W) {
                const uint2 v = *reinterpret_cast<const uint2*>(x + (((size_t)n * H + hi) * W + wi) * 4);
                xin[0] = bf16_to_f32(v.x & 0xffff);
                xin[1] = bf16_to_f32(v.x >> 16);
                xin[2] = bf16_to_f32(v.y & 0xffff);
            }
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float* wr = &sw[(kh * 3 + kw) * 4 + c][cb];
#pragma unroll
                for (int co = 0; co < 16; co++) acc[co] = fmaf(xin[c], wr[co], acc[co]);
            }
        }
    }
    uint16_t* out = y + (size_t)pix * 64 + cb;
#pragma unroll
    for (int co = 0; co < 16; co += 8) {
        uint4 o;
        o.x = (uint32_t)f32_to_bf16(fmaxf(acc[co + 0], 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(acc[co + 1], 0.f)) << 16);
        o.y = (uint32_t)f32_to_bf16(fmaxf(acc[co + 2], 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(acc[co + 3], 0.f)) << 16);
        o.z = (uint32_t)f32_to_bf16(fmaxf(acc[co + 4], 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(acc[co + 5], 0.f)) << 16);
        o.w = (uint32_t)f32_to_bf16(fmaxf(acc[co + 6], 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(acc[co + 7], 0.f)) << 16);
        *reinterpret_cast<uint4*>(out + co) = o;
    }
}

// MFMA stem: the same conv as implicit GEMM on v_mfma_f32_16x16x32_bf16.
// K = 9 taps x 4 channels = 36, padded to 64 (two K=32 steps; tap 8 alone in the
// second).  A workgroup computes two output rows (2*WO pixels x 64 couts): the
// five input rows they need are staged in LDS (1-pixel zero border), weights are
// converted once into bf16 A fragments held in registers, BN bias + ReLU fused.
template <int WO>
__global__ __launch_bounds__(256) void stem_mfma_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                        int H, int Ho, long n_tiles) {
    constexpr int W = 2 * WO;   // input width
    constexpr int LW = W + 2;   // staged row (pixels) with the zero border
    constexpr int P = 2 * WO;   // output pixels per tile
    static_assert(P % 64 == 0, "two output rows must split into 16-pixel tiles per wave");
    constexpr int PTW = P / 64;
    __shared__ uint2 sx[5 * LW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
    const int tiles = Ho / 2;
    // A row r of cout tile c holds cout (r >> 2) * 16 + 4c + (r & 3), so lane group g
    // ends up owning the 16 consecutive couts 16g .. 16g+15 of its pixel: 2 x 16-B
    // stores per pixel instead of 4 x 8 B.  Fragments are built once per
    // (persistent) workgroup.
    bf16x8 afr[4][2];
    float4 b4[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int r = lane & 15, co = (r >> 2) * 16 + 4 * c + (r & 3);
#pragma unroll
        for (int kc = 0; kc < 2; kc++) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = kc * 32 + g * 8 + j, tap = k >> 2, ch = k & 3;
                afr[c][kc][j] = (__bf16)(tap < 9 ? w[(co * 9 + tap) * 4 + ch] : 0.f);
            }
        }
        b4[c] = *reinterpret_cast<const float4*>(bias + g * 16 + 4 * c);
    }
    for (long t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const int n = (int)(t / tiles), ho0 = (int)(t - (long)n * tiles) * 2;
        const uint2* xin = reinterpret_cast<const uint2*>(x) + (size_t)n * H * W;
        __syncthreads();  // the previous tile's reads of sx are done
        for (int i = tid; i < 5 * LW; i += 256) {
            const int r = i / LW, c = i - r * LW;
            const int hi = 2 * ho0 - 1 + r, wi = c - 1;
            sx[i] = (hi >= 0 && hi < H && wi >= 0 && wi < W) ? xin[(size_t)hi * W + wi] : uint2{0u, 0u};
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PTW; i++) {
            const int pix = (wave * PTW + i) * 16 + (lane & 15);
            const int orow = pix / WO, ocol = pix - (pix / WO) * WO;
            auto tap_px = [&](int tap) { return sx[(2 * orow + tap / 3) * LW + 2 * ocol + tap % 3]; };
            const uint2 t0 = tap_px(2 * g), t1 = tap_px(2 * g + 1);
            const uint2 t8 = g == 0 ? tap_px(8) : uint2{0u, 0u};
            union {
                uint4 u;
                bf16x8 v;
            } b0, b1;
            b0.u = uint4{t0.x, t0.y, t1.x, t1.y};
            b1.u = uint4{t8.x, t8.y, 0u, 0u};
            f32x4 acc[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[c][0], b0.v, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[c][1], b1.v, acc[c], 0, 0, 0);
            }
            uint32_t o[8];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const float v0 = fmaxf(acc[c][0] + b4[c].x, 0.f), v1 = fmaxf(acc[c][1] + b4[c].y, 0.f);
                const float v2 = fmaxf(acc[c][2] + b4[c].z, 0.f), v3 = fmaxf(acc[c][3] + b4[c].w, 0.f);
                o[2 * c] = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                o[2 * c + 1] = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
            }
            uint16_t* out = y + (((size_t)n * Ho + ho0 + orow) * WO + ocol) * 64 + g * 16;
            *reinterpret_cast<uint4*>(out) = uint4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<uint4*>(out + 8) = uint4{o[4], o[5], o[6], o[7]};
        }
    }
}

// ---------------------------------------------------------------- fuse sum
// out = act(sum_k nearest_up(in[k], 2^lg[k])), one 16-B channel chunk per lane, f32 sums
// in input order.  One grid row per crop and 32-bit in-crop indices with power-of-two
// chunk counts and upsample factors as shifts: the 64-bit divisions of a flat index
// (5 per lane) made the 64x48 fuse VALU-bound.
struct FuseParams {
    const uint16_t* in[4];
    int lg[4];
    int n_in;
    uint16_t* out;
    int H, W, C, lgc, relu;
};

// out = relu(sum_k up(in_k)) per 16-B chunk, the input count a template parameter: all NI
// 16-B loads issue before the first sum (a runtime-count loop waited for each load in turn:
// +0.45 % frames/s, round 2); sums in input order
template <int NI>
__global__ __launch_bounds__(256) void fuse_sum_n_kernel(FuseParams p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    const int hw = p.H * p.W;
    if (i >= (hw << p.lgc)) return;
    const int ch = i & ((1 << p.lgc) - 1);
    const int pix = i >> p.lgc;
    const int h = (int)((unsigned)pix / (unsigned)p.W), w = pix - h * p.W;
    uint4 v[NI];
#pragma unroll
    for (int k = 0; k < NI; k++) {
        const int lg = p.lg[k];
        const int hs = p.H >> lg, ws = p.W >> lg;
        const long src = ((long)n * hs * ws + (h >> lg) * ws + (w >> lg)) * p.C + ch * 8;
        v[k] = *reinterpret_cast<const uint4*>(p.in[k] + src);
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NI; k++) {
        acc[0] += bf16_to_f32(v[k].x & 0xffff);
        acc[1] += bf16_to_f32(v[k].x >> 16);
        acc[2] += bf16_to_f32(v[k].y & 0xffff);
        acc[3] += bf16_to_f32(v[k].y >> 16);
        acc[4] += bf16_to_f32(v[k].z & 0xffff);
        acc[5] += bf16_to_f32(v[k].z >> 16);
        acc[6] += bf16_to_f32(v[k].w & 0xffff);
        acc[7] += bf16_to_f32(v[k].w >> 16);
    }
    if (p.relu)
#pragma unroll
        for (int q = 0; q < 8; q++) acc[q] = fmaxf(acc[q], 0.f);
    uint4 o;
    o.x = (uint32_t)f32_to_bf16(acc[0]) | ((uint32_t)f32_to_bf16(acc[1]) << 16);
    o.y = (uint32_t)f32_to_bf16(acc[2]) | ((uint32_t)f32_to_bf16(acc[3]) << 16);
    o.z = (uint32_t)f32_to_bf16(acc[4]) | ((uint32_t)f32_to_bf16(acc[5]) << 16);
    o.w = (uint32_t)f32_to_bf16(acc[6]) | ((uint32_t)f32_to_bf16(acc[7]) << 16);
    *reinterpret_cast<uint4*>(p.out + ((long)n * hw + pix) * p.C + ch * 8) = o;
}

}  // namespace

const uint16_t* conv_zero_region() { return zero_page(); }

int conv_cout_pad(int cout) { return cout <= 32 ? 32 : ((cout + 63) / 64) * 64; }

void launch_conv_impl(const ConvLaunch& c, hipStream_t s, bool generic_only) {
    MVP_REQUIRE(c.Cin % 32 == 0, "conv: Cin=%d must be a multiple of 32", c.Cin);
    MVP_REQUIRE(c.ks == 1 || c.ks == 3, "conv: ks=%d", c.ks);
    MVP_REQUIRE(c.stride == 1 || c.stride == 2, "conv: stride=%d", c.stride);
    MVP_REQUIRE(c.out_f32_nchw || c.Cout % 4 == 0, "conv: Cout=%d must be a multiple of 4", c.Cout);
    ConvParams p{};
    p.x = c.x;
    p.w = c.w;
    p.bias = c.bias;
    p.res = c.res;
    p.y = c.y;
    p.yf = c.yf;
    p.N = c.N;
    p.H = c.H;
    p.W = c.W;
    p.Cin = c.Cin;
    p.xs = c.x_stride ? c.x_stride : c.Cin;
    p.ys = c.y_stride ? c.y_stride : c.Cout;
    p.rs = c.r_stride ? c.r_stride : c.Cout;
    const int pad = c.ks / 2;
    p.Ho = (c.H + 2 * pad - c.ks) / c.stride + 1;
    p.Wo = (c.W + 2 * pad - c.ks) / c.stride + 1;
    p.Cout = c.Cout;
    p.Cout_pad = conv_cout_pad(c.Cout);
    p.relu = c.relu;
    p.out_f32 = c.out_f32_nchw;
    if (c.N == 0) return;
    if (generic_only) {
        MVP_REQUIRE(!c.x2 && !c.out_f32_nchw, "conv: the generic path takes one bf16 input and output");
        goto generic;
    }
    if (c.x2) {  // graph cat-fusion: only the direct 1x1 kernel reads two inputs
        MVP_REQUIRE(c.ks == 1 && launch_conv1x1_direct(c, s), "conv: dual-input conv needs the 1x1 kernel");
        MVP_HIP(hipGetLastError());
        return;
    }
    if (launch_head1x1(c, s) || launch_conv1x1_direct(c, s) || launch_tconv(c, s) ||
        launch_s2conv(c, s)) {
        MVP_HIP(hipGetLastError());
        return;
    }
generic:
    if (c.ks == 3 && c.stride == 1)
        launch_plane<3, 1>(p, s);
    else if (c.ks == 3 && c.stride == 2)
        launch_plane<3, 2>(p, s);
    else if (c.ks == 1 && c.stride == 1)
        launch_plane<1, 1>(p, s);
    else
        fail(MVP_ERR_ARG, "conv: unsupported ks=%d stride=%d", c.ks, c.stride);
    MVP_HIP(hipGetLastError());
}

void launch_conv(const ConvLaunch& c, hipStream_t s) {
    MVP_REQUIRE(!c.x_stride && !c.y_stride && !c.r_stride && c.relu != 2, "conv: views / SiLU need launch_conv_generic");
    launch_conv_impl(c, s, false);
}

void launch_conv_generic(const ConvLaunch& c, hipStream_t s) { launch_conv_impl(c, s, true); }

void launch_stem(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W,
                 hipStream_t s) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const long total = (long)N * Ho * Wo * 4;
    if (total == 0) return;
    if (Wo == 96 && H % 2 == 0 && Ho % 2 == 0) {  // the 256x192 crop: MFMA path
        static int cus = 0;
        if (cus == 0) {
            int dev = 0;
            MVP_HIP(hipGetDevice(&dev));
            MVP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        }
        const long n_tiles = (long)N * Ho / 2;
        const long grid = std::min<long>(n_tiles, (long)cus * 8);
        hipLaunchKernelGGL(stem_mfma_kernel<96>, dim3((unsigned)grid), dim3(256), 0, s, x, w, bias, y, H, Ho,
                           n_tiles);
        MVP_HIP(hipGetLastError());
        return;
    }
    hipLaunchKernelGGL(stem_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, w, bias, y, N, H, W,
                       Ho, Wo);
    MVP_HIP(hipGetLastError());
}

void launch_fuse_sum(const uint16_t* const* in, const int* up, int n_in, uint16_t* out, int N, int H, int W, int C,
                     int relu, hipStream_t s) {
    MVP_REQUIRE(n_in >= 1 && n_in <= 4, "fuse: n_in=%d", n_in);
    const int chunks = C / 8;
    MVP_REQUIRE(C % 8 == 0 && (chunks & (chunks - 1)) == 0, "fuse: C=%d (C/8 must be a power of two)", C);
    FuseParams p{};
    for (int k = 0; k < n_in; k++) {
        int lg = 0;
        while ((1 << lg) < up[k]) lg++;
        MVP_REQUIRE(up[k] == (1 << lg) && H % up[k] == 0 && W % up[k] == 0, "fuse: bad upsample factor %d", up[k]);
        p.in[k] = in[k];
        p.lg[k] = lg;
    }
    int lgc = 0;
    while ((1 << lgc) < chunks) lgc++;
    p.n_in = n_in;
    p.out = out;
    p.H = H;
    p.W = W;
    p.C = C;
    p.lgc = lgc;
    p.relu = relu;
    const long per = (long)H * W * chunks;
    MVP_REQUIRE(per < (1L << 30) && N < 65536, "fuse: plane too large");
    if (per == 0 || N == 0) return;
    const dim3 g((unsigned)((per + 255) / 256), (unsigned)N);
    if (n_in == 1)
        hipLaunchKernelGGL(fuse_sum_n_kernel<1>, g, dim3(256), 0, s, p);
    else if (n_in == 2)
        hipLaunchKernelGGL(fuse_sum_n_kernel<2>, g, dim3(256), 0, s, p);
    else if (n_in == 3)
        hipLaunchKernelGGL(fuse_sum_n_kernel<3>, g, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL(fuse_sum_n_kernel<4>, g, dim3(256), 0, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
