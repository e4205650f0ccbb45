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

bool launch_conv1x1_direct(const ConvLaunch& c, hipStream_t s) {
    if (c.ks != 1 || c.stride != 1 || c.out_f32_nchw || c.Cin % 32 != 0) return false;
    const int bm = conv_cout_pad(c.Cout) % 128 == 0 && c.Cin <= 64 ? 128 : conv_cout_pad(c.Cout) % 64 == 0 ? 64 : 32;
    if (c.Cout % (bm / 4) != 0) return false;  // lane groups own bm/4 consecutive couts
    static const bool disabled = [] {
        const char* e = getenv("MVPOSE_NO_1X1");  // diagnostics: use the generic conv kernel
        return e && e[0] == '1';
    }();
    if (disabled && !c.x2) return false;
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
