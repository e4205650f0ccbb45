// Fused HRNet BasicBlock for the 32-channel, full-width branch (64x48 planes):
//   y = relu( conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x )
// in ONE kernel: the intermediate activation never leaves LDS and the residual is
// the centre of the input halo already staged for conv1.  Against two separate
// convs this removes the intermediate's HBM write + read and the residual re-read
// (5 tensor passes -> 2), the layer being HBM-bound on MI355X.
//
// Persistent workgroups of 8 waves walk tiles of 8 output rows x W columns of one
// crop.  Per tile:
//   input halo  (8+4) x (W+4) pixels x 32 ch, LDS-DMA double-buffered (the next
//               tile's halo streams in under this tile's MFMAs)
//   conv1       on the (8+2) x (W+2) ring it feeds conv2 (recomputed border);
//               outside the image the intermediate is 0 (conv2's zero padding)
//   conv2       8 x W outputs, + bias + residual (LDS) + ReLU -> bf16 NHWC
// Same MFMA (v_mfma_f32_16x16x32_bf16), same K order (taps 0..8, one 32-channel
// chunk) and same epilogue arithmetic as conv_mfma_kernel, so the result is
// bit-identical to running the two convs separately.
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

// s_waitcnt lgkmcnt(n) alone (vmcnt / expcnt at their maxima), visible to the
// compiler's wait-count pass: waiting for all but the n youngest LDS reads lets a
// tap's MFMAs start while the next tap's fragments are still in flight.
template <int n>
__device__ __forceinline__ void wait_lgkm() {
    static_assert(n >= 0 && n < 16, "lgkmcnt is 4 bits");
    __builtin_amdgcn_s_waitcnt(0xC07F | (n << 8));
}

__device__ __forceinline__ float bf16_to_f32(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}

template <int W>
struct BlockCfg {
    static constexpr int NW = 8, NT = NW * 64;
    static constexpr int TH = 8;
    static constexpr int XH = TH + 4, XW = W + 4;   // input halo
    static constexpr int MH = TH + 2, MW = W + 2;   // conv1 ring (intermediate)
    static constexpr int XPIX = XH * XW, MPIX = MH * MW, OPIX = TH * W;
    static constexpr int XP = (XPIX + 127) / 128 * 128;   // per chunk plane, whole pieces for 8 waves
    static constexpr int MP = (MPIX + 15) / 16 * 16;
    static constexpr int X_BYTES = 4 * XP * 16;
    static constexpr int M_BYTES = 4 * MP * 16;
    static constexpr int W_SLOTS = 9 * 4 * 32;            // one conv's [tap][q][cout] slice
    static constexpr int W_BYTES = W_SLOTS * 16;
    static constexpr int LDS = 2 * X_BYTES + M_BYTES + 2 * W_BYTES;
    static constexpr int PT1 = MP / 16 / NW;              // conv1 pixel tiles per wave
    static constexpr int PT2 = OPIX / 16 / NW;            // conv2 pixel tiles per wave
    static constexpr int X_OPS = 4 * XP / NT;             // halo DMA pieces per wave
    static_assert((MP / 16) % NW == 0 && (OPIX / 16) % NW == 0, "tiles must split over the waves");
    static_assert((4 * XP) % NT == 0, "halo must split into whole pieces");
};

struct BlockParams {
    const uint16_t* x;
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    uint16_t* y;
    const uint16_t* zero;  // >= 64 KiB of zeros
    int N, H, n_tiles;
};

template <int W>
__global__ __launch_bounds__(512, 2) void basic_block_c32_kernel(BlockParams p) {
    using C = BlockCfg<W>;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    __shared__ float4 sb1[8], sb2[8];
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= p.n_tiles) return;
    uint8_t* xbuf0 = lds;
    uint8_t* mbuf = lds + 2 * C::X_BYTES;
    uint8_t* wbuf1 = mbuf + C::M_BYTES;
    uint8_t* wbuf2 = wbuf1 + C::W_BYTES;
    const int H = p.H, tiles_h = H / C::TH;
    const size_t plane = (size_t)H * W;
    if (tid < 8) {
        sb1[tid] = reinterpret_cast<const float4*>(p.b1)[tid];
        sb2[tid] = reinterpret_cast<const float4*>(p.b2)[tid];
    }

    // ---- weights (both convs) straight into LDS, [tap][q][cout] slots
    for (int s0 = wave * 64; s0 < C::W_SLOTS; s0 += C::NT) {
        const int sl = s0 + lane, co = sl & 31, tq = sl >> 5;  // tq = tap * 4 + q
        const size_t off = ((size_t)co * 9 + (tq >> 2)) * 32 + (tq & 3) * 8;
        glds16(p.w1 + off, wbuf1 + s0 * 16);
        glds16(p.w2 + off, wbuf2 + s0 * 16);
    }

    // ---- per-lane halo geometry of this wave's DMA pieces
    int hgeo[C::X_OPS], hoff[C::X_OPS];
#pragma unroll
    for (int j = 0; j < C::X_OPS; j++) {
        const int sw0 = j * C::NT + wave * 64;
        const int q = sw0 / C::XP, pix = sw0 - q * C::XP + lane;
        const int hr = pix / C::XW, hc = pix - (pix / C::XW) * C::XW;
        hgeo[j] = pix < C::XPIX ? (hr | (hc << 10)) : -1;
        hoff[j] = (hr * W + hc) * 32 + q * 8;
    }
    auto issue = [&](int k, uint8_t* xb) {
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, ho0 = (tile - n * tiles_h) * C::TH;
        const int hi0 = ho0 - 2, wi0 = -2;
        const uint16_t* base = p.x + ((long)n * (long)plane + (long)hi0 * W + wi0) * 32;
#pragma unroll
        for (int j = 0; j < C::X_OPS; j++) {
            const int sw0 = j * C::NT + wave * 64;
            const int gg = hgeo[j];
            const int hr = gg & 1023, hc = gg >> 10;
            const bool in = gg >= 0 && n < p.N && (unsigned)(hi0 + hr) < (unsigned)H && (unsigned)(wi0 + hc) < (unsigned)W;
            const void* src = in ? (const void*)(base + hoff[j]) : (const void*)(p.zero + ((sw0 + lane) & 4095) * 8);
            glds16(src, xb + sw0 * 16);
        }
    };

    // fragment bases: B reads pixel (lane & 15) of a 16-pixel tile, chunk q = lane >> 4
    int b1base[C::PT1], b2base[C::PT2], m1pix[C::PT1];
#pragma unroll
    for (int i = 0; i < C::PT1; i++) {
        int m = (wave * C::PT1 + i) * 16 + (lane & 15);
        m1pix[i] = m;
        if (m >= C::MPIX) m = C::MPIX - 1;  // padding pixels: computed, never written
        const int r = m / C::MW, c = m - (m / C::MW) * C::MW;
        b1base[i] = (g * C::XP + r * C::XW + c) * 16;
    }
#pragma unroll
    for (int i = 0; i < C::PT2; i++) {
        const int pp = (wave * C::PT2 + i) * 16 + (lane & 15);
        const int r = pp / W, c = pp - (pp / W) * W;
        b2base[i] = (g * C::MP + r * C::MW + c) * 16;
    }
    const int abase = (g * 32 + (lane & 15)) * 16;

    const int n_items = (p.n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    issue(0, xbuf0);
    int buf = 0;
    for (int k = 0; k < n_items; k++) {
        // this wave's pieces of tile k landed (first tile: also the weights); only the
        // stores of tile k-1 (PT2 x 2 per wave) are younger
        if (k == 0)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::PT2 * 2) : "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        uint8_t* xb = xbuf0 + buf * C::X_BYTES;
        issue(k + 1, xbuf0 + (buf ^ 1) * C::X_BYTES);  // past the end: zero-region reads, never used
        const int tile = blockIdx.x + k * gridDim.x;
        const int n = tile / tiles_h, ho0 = (tile - n * tiles_h) * C::TH;

        // ---- conv1 on the (TH+2) x (W+2) ring
        {
            f32x4 acc[C::PT1][2];
#pragma unroll
            for (int i = 0; i < C::PT1; i++) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            // fragments of tap t+1 load under tap t's MFMAs (two register sets)
            bf16x8 fa[2][2], fb[2][C::PT1];
            auto load1 = [&](int tap, bf16x8 (&a)[2], bf16x8 (&b)[C::PT1]) {
                const int toff = ((tap / 3) * C::XW + tap % 3) * 16;
#pragma unroll
                for (int c = 0; c < 2; c++)
                    a[c] = *reinterpret_cast<const bf16x8*>(wbuf1 + tap * 4 * 32 * 16 + abase + c * 256);
#pragma unroll
                for (int i = 0; i < C::PT1; i++) b[i] = *reinterpret_cast<const bf16x8*>(xb + b1base[i] + toff);
            };
            load1(0, fa[0], fb[0]);
#pragma unroll
            for (int tap = 0; tap < 9; tap++) {
                const int cur = tap & 1;
                if (tap + 1 < 9) load1(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
                __builtin_amdgcn_sched_barrier(0);
                if (tap + 1 < 9)
                    wait_lgkm<2 + C::PT1>();
                else
                    wait_lgkm<0>();
#pragma unroll
                for (int i = 0; i < C::PT1; i++)
#pragma unroll
                    for (int c = 0; c < 2; c++)
                        acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][c], fb[cur][i], acc[i][c], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < C::PT1; i++) {
                const int m = m1pix[i];
                if (m >= C::MPIX) continue;
                const int r = m / C::MW, c = m - (m / C::MW) * C::MW;
                const bool inside = (unsigned)(ho0 - 1 + r) < (unsigned)H && (unsigned)(c - 1) < (unsigned)W;
#pragma unroll
                for (int ct = 0; ct < 2; ct++) {
                    const float4 bb = sb1[ct * 4 + g];
                    const float v0 = fmaxf(acc[i][ct][0] + bb.x, 0.f), v1 = fmaxf(acc[i][ct][1] + bb.y, 0.f);
                    const float v2 = fmaxf(acc[i][ct][2] + bb.z, 0.f), v3 = fmaxf(acc[i][ct][3] + bb.w, 0.f);
                    uint2 o;
                    o.x = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                    o.y = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
                    if (!inside) o = uint2{0u, 0u};
                    // couts 16ct + 4g .. +3 -> chunk q = 2ct + g/2, byte (g & 1) * 8 of the pixel's slot
                    *reinterpret_cast<uint2*>(mbuf + ((2 * ct + (g >> 1)) * C::MP + m) * 16 + (g & 1) * 8) = o;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");

        // ---- conv2 on the TH x W outputs, + bias + residual + ReLU
        {
            f32x4 acc[C::PT2][2];
#pragma unroll
            for (int i = 0; i < C::PT2; i++) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            bf16x8 fa[2][2], fb[2][C::PT2];
            auto load2 = [&](int tap, bf16x8 (&a)[2], bf16x8 (&b)[C::PT2]) {
                const int toff = ((tap / 3) * C::MW + tap % 3) * 16;
#pragma unroll
                for (int c = 0; c < 2; c++)
                    a[c] = *reinterpret_cast<const bf16x8*>(wbuf2 + tap * 4 * 32 * 16 + abase + c * 256);
#pragma unroll
                for (int i = 0; i < C::PT2; i++) b[i] = *reinterpret_cast<const bf16x8*>(mbuf + b2base[i] + toff);
            };
            load2(0, fa[0], fb[0]);
#pragma unroll
            for (int tap = 0; tap < 9; tap++) {
                const int cur = tap & 1;
                if (tap + 1 < 9) load2(tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
                __builtin_amdgcn_sched_barrier(0);
                if (tap + 1 < 9)
                    wait_lgkm<2 + C::PT2>();
                else
                    wait_lgkm<0>();
#pragma unroll
                for (int i = 0; i < C::PT2; i++)
#pragma unroll
                    for (int c = 0; c < 2; c++)
                        acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][c], fb[cur][i], acc[i][c], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            const bool valid_n = n < p.N;
#pragma unroll
            for (int i = 0; i < C::PT2; i++) {
                const int pp = (wave * C::PT2 + i) * 16 + (lane & 15);
                const int r = pp / W, c = pp - (pp / W) * W;
                uint16_t* yrow = p.y + (((size_t)n * H + ho0 + r) * W + c) * 32;
#pragma unroll
                for (int ct = 0; ct < 2; ct++) {
                    const float4 bb = sb2[ct * 4 + g];
                    float v0 = acc[i][ct][0] + bb.x, v1 = acc[i][ct][1] + bb.y;
                    float v2 = acc[i][ct][2] + bb.z, v3 = acc[i][ct][3] + bb.w;
                    const uint2 rv = *reinterpret_cast<const uint2*>(
                        xb + ((2 * ct + (g >> 1)) * C::XP + (r + 2) * C::XW + c + 2) * 16 + (g & 1) * 8);
                    v0 += bf16_to_f32(rv.x & 0xffff);
                    v1 += bf16_to_f32(rv.x >> 16);
                    v2 += bf16_to_f32(rv.y & 0xffff);
                    v3 += bf16_to_f32(rv.y >> 16);
                    uint2 o;
                    o.x = (uint32_t)f32_to_bf16(fmaxf(v0, 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(v1, 0.f)) << 16);
                    o.y = (uint32_t)f32_to_bf16(fmaxf(v2, 0.f)) | ((uint32_t)f32_to_bf16(fmaxf(v3, 0.f)) << 16);
                    // every store issues (the vmcnt accounting above counts them); a tile past
                    // the last crop cannot occur (k < n_items), so valid_n is always true here
                    uint16_t* dst = valid_n ? yrow + ct * 16 + g * 4 : const_cast<uint16_t*>(p.zero);
                    *reinterpret_cast<uint2*>(dst) = o;
                }
            }
        }
        buf ^= 1;
    }
}

int g_cus = 0;

}  // namespace

bool basic_block_c32_supported(int H, int W) { return W == 48 && H % 8 == 0; }

void launch_basic_block_c32(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2,
                            const float* b2, uint16_t* y, int N, int H, int W, hipStream_t s) {
    MVP_REQUIRE(basic_block_c32_supported(H, W), "basic block: unsupported plane %dx%d", H, W);
    if (N == 0) return;
    if (launch_tblock32s(x, w1, b1, w2, b2, y, N, H, W, s)) return;  // streaming version (tblock32s.hip)
    if (launch_tblock32(x, w1, b1, w2, b2, y, N, H, W, s)) return;   // tile version (tblock.hip)
    using C = BlockCfg<48>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)basic_block_c32_kernel<48>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
        attr = true;
    }
    if (g_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    BlockParams p{x, w1, b1, w2, b2, y, conv_zero_region(), N, H, (int)((long)N * (H / C::TH))};
    const int grid = std::min(p.n_tiles, g_cus);
    hipLaunchKernelGGL(basic_block_c32_kernel<48>, dim3(grid), dim3(C::NT), C::LDS, s, p);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp
