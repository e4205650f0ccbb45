// Person detector (RTMDet-m) kernels for gfx950: the parts of the network that are not
// dense convolutions (those run on conv_mfma_kernel through launch_conv_generic), plus
// the test pipeline in front of it and the prediction / selection behind it.
//
// Reference: PoseEstimator.predict -> mmdet inference_detector (mmpose_pose_estimation.py
// :98-99, :234-241) and the hand-off rule (:242-250); algorithm restated in
// oracle/rtmdet_ref.py (mmdet / mmcv / cv2 are absent here: parity unpinned).
//
// Layout: bf16 NHWC activations; a "view" is a channel slice [coff, coff + c) of a
// tensor whose pixels are `stride` elements apart, so concatenation is free (producers
// write into their slice of the shared buffer).
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "conv.h"
#include "det.h"
#include "mvp_common.h"

#ifndef DET_HALO_TR
#define DET_HALO_TR 4  // output rows per halo tile (2, 4 or 8)
#endif

namespace mvp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf(uint32_t v16) { return __uint_as_float(v16 << 16); }
__device__ __forceinline__ uint32_t tobf(float f) {
    __bf16 b = (__bf16)f;  // round to nearest even
    return (uint32_t)__builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float act_f(float v, int act) {
    if (act == 1) return fmaxf(v, 0.f);
    if (act == 2) return v * __builtin_amdgcn_rcpf(1.f + __expf(-v));  // v_exp + v_rcp (1 ulp): output is bf16
    return v;
}
__device__ __forceinline__ void unpack8(uint4 u, float* f) {
    f[0] = bf(u.x & 0xffff), f[1] = bf(u.x >> 16), f[2] = bf(u.y & 0xffff), f[3] = bf(u.y >> 16);
    f[4] = bf(u.z & 0xffff), f[5] = bf(u.z >> 16), f[6] = bf(u.w & 0xffff), f[7] = bf(u.w >> 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    return uint4{tobf(f[0]) | (tobf(f[1]) << 16), tobf(f[2]) | (tobf(f[3]) << 16), tobf(f[4]) | (tobf(f[5]) << 16),
                 tobf(f[6]) | (tobf(f[7]) << 16)};
}

// ------------------------------------------------------------------ letterbox
// One thread per output pixel.  cv2.resize INTER_LINEAR on uint8 (OpenCV 4.x
// imgproc/resize.cpp): an exact 2x downscale runs INTER_AREA's fast path,
// (a + b + c + d + 2) >> 2; otherwise fixed-point bilinear with 11-bit coefficients,
// exact int32 horizontal pass and the SIMD vertical rounding
// (((S0 >> 4) * b0 >> 16) + ((S1 >> 4) * b1 >> 16) + 2) >> 2.
struct LbParams {
    const uint8_t* f;
    uint32_t* out;  // [n][S][S] pixels of 4 bf16 (8 B = 2 words)
    int H, W, S, nh, nw, area2;
    double scale_x, scale_y;
    float mean[3], stdv[3];
};

__device__ __forceinline__ void lin_coef(int d, double scale, int n_src, int& s0, int& s1, int& c0, int& c1) {
    float fx = (float)((d + 0.5) * scale - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) fx = 0.f, sx = 0;
    if (sx >= n_src - 1) fx = 0.f, sx = n_src - 1;
    c1 = (int)rintf(fx * 2048.f);
    c0 = (int)rintf((1.f - fx) * 2048.f);
    s0 = sx;
    s1 = min(sx + 1, n_src - 1);
}

// normalised bf16 channels of a letterboxed u8 pixel (+ a zero 4th)
__device__ __forceinline__ uint2 lb_pack(const LbParams& p, const int* v) {
    float o[3];
#pragma unroll
    for (int c = 0; c < 3; c++) o[c] = ((float)v[c] - p.mean[c]) / p.stdv[c];
    return uint2{tobf(o[0]) | (tobf(o[1]) << 16), tobf(o[2])};
}

// the u8 channels of letterboxed pixel (y, x) of frame n (114 in the padding)
__device__ __forceinline__ void lb_u8(const LbParams& p, int n, int y, int x, int* v) {
    v[0] = v[1] = v[2] = 114;
    const uint8_t* fr = p.f + (size_t)n * p.H * p.W * 3;
    if (y < p.nh && x < p.nw) {
        if (p.area2) {
            const uint8_t* r0 = fr + ((size_t)(2 * y) * p.W + 2 * x) * 3;
            const uint8_t* r1 = r0 + (size_t)p.W * 3;
#pragma unroll
            for (int c = 0; c < 3; c++) v[c] = (r0[c] + r0[3 + c] + r1[c] + r1[3 + c] + 2) >> 2;
        } else {
            int x0, x1, a0, a1, y0, y1, b0, b1;
            lin_coef(x, p.scale_x, p.W, x0, x1, a0, a1);
            lin_coef(y, p.scale_y, p.H, y0, y1, b0, b1);
            const uint8_t* r0 = fr + (size_t)y0 * p.W * 3;
            const uint8_t* r1 = fr + (size_t)y1 * p.W * 3;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const int h0 = r0[x0 * 3 + c] * a0 + r0[x1 * 3 + c] * a1;
                const int h1 = r1[x0 * 3 + c] * a0 + r1[x1 * 3 + c] * a1;
                const int s = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
                v[c] = min(max((s + 2) >> 2, 0), 255);
            }
        }
    }
}

// letterboxed pixel (y, x) of frame n: 3 normalised bf16 channels + a zero 4th
__device__ __forceinline__ uint2 lb_pixel(const LbParams& p, int n, int y, int x) {
    int v[3];
    lb_u8(p, n, y, x, v);
    return lb_pack(p, v);
}

// lb_pack through a table of the 3 x 256 normalised values (the stem's staging: the same
// division, done once per value instead of three times per pixel)
__device__ __forceinline__ uint2 lb_pack_lut(const uint16_t* lut, const int* v) {
    return uint2{(uint32_t)lut[v[0]] | ((uint32_t)lut[256 + v[1]] << 16), (uint32_t)lut[512 + v[2]]};
}

// letterboxed pixels (y, x) and (y, x + 1), x even, of frame n on the INTER_AREA fast path (the
// stem's staging, round 6): their 2 x 2 source blocks are 12 contiguous bytes per source row,
// read as 3 dwords instead of 12 bytes each (needs the row start 4-byte aligned: W % 4 == 0);
// the same integer arithmetic as lb_pixel
__device__ __forceinline__ void lb_pair(const LbParams& p, int n, int y, int x, uint2& o0, uint2& o1,
                                        const uint16_t* lut) {
    if (!p.area2 || (p.W & 3) || y >= p.nh || x + 1 >= p.nw) {
        int v0[3], v1[3];
        lb_u8(p, n, y, x, v0);
        lb_u8(p, n, y, x + 1, v1);
        o0 = lb_pack_lut(lut, v0);
        o1 = lb_pack_lut(lut, v1);
        return;
    }
    const uint8_t* r0 = p.f + ((size_t)n * p.H * p.W + (size_t)(2 * y) * p.W + 2 * x) * 3;
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(r0);
    const uint32_t* w1 = reinterpret_cast<const uint32_t*>(r0 + (size_t)p.W * 3);
    const uint32_t a[3] = {w0[0], w0[1], w0[2]}, b[3] = {w1[0], w1[1], w1[2]};
    auto byte = [](const uint32_t* w, int i) { return (int)((w[i >> 2] >> ((i & 3) * 8)) & 0xff); };
    int v0[3], v1[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        v0[c] = (byte(a, c) + byte(a, 3 + c) + byte(b, c) + byte(b, 3 + c) + 2) >> 2;
        v1[c] = (byte(a, 6 + c) + byte(a, 9 + c) + byte(b, 6 + c) + byte(b, 9 + c) + 2) >> 2;
    }
    o0 = lb_pack_lut(lut, v0);
    o1 = lb_pack_lut(lut, v1);
}

__global__ __launch_bounds__(256) void letterbox_kernel(LbParams p) {
    const int n = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.S * p.S) return;
    const int y = i / p.S, x = i - y * p.S;
    *reinterpret_cast<uint2*>(p.out + ((size_t)n * p.S * p.S + i) * 2) = lb_pixel(p, n, y, x);
}

// ------------------------------------------------------------------ stem conv
// 3x3/s2 conv 4 -> 32 channels (24 real + zero-weight padding) on v_mfma_f32_16x16x32_bf16:
// K = 9 taps x 4 channels = 36 padded to 64.  A workgroup computes two output rows; the
// five input rows they read are staged in LDS with a one-pixel zero border.  A row r of
// cout tile c is cout (r >> 2) * 8 + 4c + (r & 3), so lane group g owns the 8 consecutive
// couts 8g..8g+7 of its pixel (one 16-B store).
// LB (round 6): the five input rows are letterboxed from the raw frames as they are staged
// (lb_pixel: letterbox_kernel's arithmetic), so the letterboxed image is never written or read
// back (the letterbox pass folded into the stem; bit-identical).
template <bool LB>
__global__ __launch_bounds__(256) void det_stem_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                       int S, int act, long n_tiles, LbParams lb) {
    extern __shared__ uint2 sx[];  // [5][S + 2]
    __shared__ uint16_t lut[LB ? 3 * 256 : 1];  // LB: the normalised bf16 of every u8 value
    const int Wo = S / 2, LW = S + 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
    if constexpr (LB)
        for (int i = tid; i < 3 * 256; i += 256) {
            const int c = i >> 8;
            lut[i] = (uint16_t)tobf(((float)(i & 255) - lb.mean[c]) / lb.stdv[c]);
        }
    bf16x8 afr[2][2];
    float4 b4[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int r = lane & 15, co = (r >> 2) * 8 + 4 * c + (r & 3);
#pragma unroll
        for (int kc = 0; kc < 2; kc++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = kc * 32 + g * 8 + j, tap = k >> 2, ch = k & 3;
                afr[c][kc][j] = (__bf16)(tap < 9 ? w[(co * 9 + tap) * 4 + ch] : 0.f);
            }
        b4[c] = *reinterpret_cast<const float4*>(bias + g * 8 + 4 * c);
    }
    const int tiles = Wo / 2;  // output row pairs per image (Ho = Wo)
    const int n_pt = Wo * 2 / 16;  // 16-pixel tiles per row pair
    for (long t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const long n = t / tiles;
        const int ho0 = (int)(t - n * tiles) * 2;
        const uint2* xin = reinterpret_cast<const uint2*>(x) + (size_t)n * S * S;
        __syncthreads();
        if constexpr (LB) {
            // pixel pairs (wi, wi + 1), wi even, of the five rows; the zero border columns apart
            const int PR = S / 2;
            for (int i = tid; i < 5 * PR; i += 256) {
                const int r = i / PR, wi = 2 * (i - r * PR);
                const int hi = 2 * ho0 - 1 + r;
                uint2 o0 = {0u, 0u}, o1 = {0u, 0u};
                if (hi >= 0 && hi < S) lb_pair(lb, (int)n, hi, wi, o0, o1, lut);
                sx[r * LW + wi + 1] = o0;
                sx[r * LW + wi + 2] = o1;
            }
            if (tid < 10) sx[(tid >> 1) * LW + (tid & 1) * (LW - 1)] = uint2{0u, 0u};
        } else {
            for (int i = tid; i < 5 * LW; i += 256) {
                const int r = i / LW, c = i - r * LW;
                const int hi = 2 * ho0 - 1 + r, wi = c - 1;
                const bool in = hi >= 0 && hi < S && wi >= 0 && wi < S;
                sx[i] = in ? xin[(size_t)hi * S + wi] : uint2{0u, 0u};
            }
        }
        __syncthreads();
        for (int pt = wave; pt < n_pt; pt += 4) {
            const int pix = pt * 16 + (lane & 15);
            const int orow = pix / Wo, ocol = pix - orow * Wo;
            auto tap_px = [&](int tap) { return sx[(2 * orow + tap / 3) * LW + 2 * ocol + tap % 3]; };
            const uint2 t0 = tap_px(2 * g), t1 = tap_px(2 * g + 1);
            const uint2 t8 = g == 0 ? tap_px(8) : uint2{0u, 0u};
            union {
                uint4 u;
                bf16x8 v;
            } q0, q1;
            q0.u = uint4{t0.x, t0.y, t1.x, t1.y};
            q1.u = uint4{t8.x, t8.y, 0u, 0u};
            uint32_t o[4];
#pragma unroll
            for (int c = 0; c < 2; c++) {
                f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[c][0], q0.v, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[c][1], q1.v, acc, 0, 0, 0);
                o[2 * c] = tobf(act_f(acc[0] + b4[c].x, act)) | (tobf(act_f(acc[1] + b4[c].y, act)) << 16);
                o[2 * c + 1] = tobf(act_f(acc[2] + b4[c].z, act)) | (tobf(act_f(acc[3] + b4[c].w, act)) << 16);
            }
            uint16_t* out = y + (((size_t)n * Wo + ho0 + orow) * Wo + ocol) * 32 + g * 8;
            *reinterpret_cast<uint4*>(out) = uint4{o[0], o[1], o[2], o[3]};
        }
    }
}

// ------------------------------------------------------------------ depthwise 5x5
// Memory-bound (25 MACs per element): one workgroup = an 8 x 16 output tile x G channel
// chunks of 8 (G waves, one chunk per wave).  The 12 x 20 input halo is loaded coalesced
// (G consecutive 16-B chunks of a pixel per lane group) into LDS stored chunk-major, so a
// wave's fragment reads are 64 consecutive pixels of its chunk (conflict-free).  Each lane
// computes two vertically adjacent outputs (6 input rows x 5 taps for 2 outputs); the
// weights are wave-uniform ([C/8][25][8] f32), read through the scalar cache.
constexpr int kDwTH = 8, kDwTW = 16, kDwHH = kDwTH + 4, kDwHW = kDwTW + 4;

struct DwParams {
    const uint16_t* x;
    uint16_t* y;
    const float* w;  // [C/8][25][8]
    const float* b;  // [C]
    int H, W, C, xs, ys, act, tiles_w;
};

template <int G>
__global__ __launch_bounds__(G * 64, 8 / G * 2) void dw5_kernel(DwParams p) {
    __shared__ uint4 sh[G][kDwHH * kDwHW];
    const int n_groups = p.C / (8 * G);
    const int grp = blockIdx.x % n_groups;
    const int t2 = blockIdx.x / n_groups;
    const int tw = t2 % p.tiles_w, th = t2 / p.tiles_w;
    const int n = blockIdx.y;
    const int h0 = th * kDwTH - 2, w0 = tw * kDwTW - 2;
    const int tid = threadIdx.x;
    const uint16_t* xb = p.x + (size_t)n * p.H * p.W * p.xs + grp * 8 * G;
    for (int i = tid; i < kDwHH * kDwHW * G; i += G * 64) {
        const int pix = i / G, q = i - pix * G;
        const int r = pix / kDwHW, c = pix - r * kDwHW;
        const int hi = h0 + r, wi = w0 + c;
        sh[q][pix] = (hi >= 0 && hi < p.H && wi >= 0 && wi < p.W)
                         ? *reinterpret_cast<const uint4*>(xb + ((size_t)hi * p.W + wi) * p.xs + q * 8)
                         : uint4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int col = lane & 15, rp = lane >> 4;
    const int chunk = grp * G + wave;
    const float* wc = p.w + (size_t)chunk * 200;
    // channel pairs on packed FMAs (v_pk_fma_f32: two fmaf per instruction, the same roundings):
    // the kernel is VALU-issue-bound (~1,100 VALU instructions per wave with scalar fmaf)
    typedef float f32x2v __attribute__((ext_vector_type(2)));
    f32x2v a0[4], a1[4];
#pragma unroll
    for (int c = 0; c < 4; c++) a0[c] = a1[c] = f32x2v{0.f, 0.f};
    // input rows one at a time (not unrolled): 8 unpacked values live, not 240, so the
    // kernel fits 8 waves per SIMD and the next block's halo load hides under this one
#pragma unroll 1
    for (int ir = 0; ir < 6; ir++) {
#pragma unroll
        for (int kw = 0; kw < 5; kw++) {
            float v[8];
            unpack8(sh[wave][(2 * rp + ir) * kDwHW + col + kw], v);
            if (ir < 5) {
                const float* wk = wc + (ir * 5 + kw) * 8;
#pragma unroll
                for (int c = 0; c < 4; c++)
                    a0[c] = __builtin_elementwise_fma(f32x2v{v[2 * c], v[2 * c + 1]},
                                                      f32x2v{wk[2 * c], wk[2 * c + 1]}, a0[c]);
            }
            if (ir >= 1) {
                const float* wk = wc + ((ir - 1) * 5 + kw) * 8;
#pragma unroll
                for (int c = 0; c < 4; c++)
                    a1[c] = __builtin_elementwise_fma(f32x2v{v[2 * c], v[2 * c + 1]},
                                                      f32x2v{wk[2 * c], wk[2 * c + 1]}, a1[c]);
            }
        }
    }
    const int ho = th * kDwTH + 2 * rp, wo = tw * kDwTW + col;
    if (wo >= p.W) return;
    const float* bc = p.b + chunk * 8;
    float o0[8], o1[8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        o0[c] = act_f(a0[c >> 1][c & 1] + bc[c], p.act);
        o1[c] = act_f(a1[c >> 1][c & 1] + bc[c], p.act);
    }
    uint16_t* yb = p.y + ((size_t)n * p.H * p.W + (size_t)ho * p.W + wo) * p.ys + chunk * 8;
    if (ho < p.H) *reinterpret_cast<uint4*>(yb) = pack8(o0);
    if (ho + 1 < p.H) *reinterpret_cast<uint4*>(yb + (size_t)p.W * p.ys) = pack8(o1);
}

// ------------------------------------------------------------------ conv = GEMM
// Every detector conv is a GEMM over the flat output-pixel index m = (n, ho, wo):
//   Y[m][cout] = sum_k X~[m][k] W[cout][k],  k = (tap, cin) (weights [cout][kh][kw][cin]),
// X~ the im2col of the NHWC input view, gathered on the fly: K step (tap, 32-channel chunk)
// DMAs, for each of the tile's 128 pixels, the 64 bytes of its tap's input pixel (or zeros
// outside the image) straight into LDS (global_load_lds); a 1x1 conv reads its own pixel.
// Flat pixels need no masking on 20x20 or 40x40 planes, and the same kernel serves the
// stride-2 downsamples.  Workgroup tile: 128 pixels x BN couts, 4 waves as 2 (pixels) x 2
// (couts), operands double-buffered chunk-major in LDS ([k group][row] 16-B slots: every
// 16-lane fragment read is 256 contiguous bytes), the next K step's DMA in flight under
// the current step's MFMAs (v_mfma_f32_16x16x32_bf16).  Epilogue: bias, activation (SiLU
// before the residual, ReLU after it), bf16 stores into the output view.  Workgroups run
// couts-fastest so the blocks sharing an input tile are co-resident (input from HBM once,
// taps from L2).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
__device__ __forceinline__ void glds16_det(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_base, 16, 0, 0);
}

struct GParams {
    const uint16_t* x;
    const uint16_t* w;  // [npad][KS*KS*cin]
    const float* bias;  // [npad]
    const uint16_t* res;
    uint16_t* y;
    const uint16_t* zero;  // >= 16 KiB of zeros
    long M;                // n * Ho * Wo
    int cin, N, npad, xs, ys, rs, act, n_nb;
    int xcd_order;         // GEMM kernel: XCD-contiguous logical block order
    int H, W, Ho, Wo;
    // GEMM kernel: w re-laid by det_pack_gemm_weights (per 32-channel K step, every cout's
    // four swizzled 16-B chunks in LDS slot order: a weight DMA instruction reads 1 KB
    // contiguous instead of 16 rows x 64 B); nullptr: gather from w
    const uint16_t* wimg = nullptr;
    // persistent 1x1 GEMM folds (DetConvFold, det.h): input channels [0, up_c) from the nearest-2x
    // upsample of `up` (an H/2 x W/2 plane, pixel stride up_s); `ca`: [n][cin] f32 channel scales
    const uint16_t* up = nullptr;
    const float* ca = nullptr;
    int up_s = 0, up_c = 0;
};

// s_waitcnt vmcnt(n') for the largest level n' <= n (wave-uniform n): at most n' of this
// wave's vector-memory operations stay outstanding (rounding down only waits longer)
__device__ __forceinline__ void wait_vm(int n) {
    if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// PW waves along the pixels (16*FP each) x 2 along the couts: tile 16*FP*PW pixels x BN couts.
// (a 2-slot ring with one chunk per step leaves LDS for three workgroups per CU; FP = 8
// holds a 128 x BN/2 accumulator tile per wave, one wave per SIMD)
template <int BN, int KS, int S, int PW, int NBUF, int CPS, int FP = 4>
__global__ __launch_bounds__(128 * PW, FP == 8 ? 1 : (PW == 2 && NBUF == 2 && CPS == 1) ? 3 : 4 / PW) void
det_conv_gemm_kernel(GParams p) {
    constexpr int NT = 128 * PW;          // threads
    constexpr int NWV = 2 * PW;           // waves
    constexpr int BMP = 16 * FP * PW;     // pixels per tile
    constexpr int A_SLOTS = 4 * BN;       // [kg][cout]
    constexpr int B_SLOTS = 4 * BMP;      // [kg][pix]
    constexpr int SUB = (A_SLOTS + B_SLOTS) * 16;  // one 32-channel K chunk
    constexpr int STAGE = CPS * SUB;      // CPS chunks per ring slot (per barrier)
    constexpr int WCT = BN / 32;          // cout tiles per wave
    constexpr int PAD = KS / 2;
    constexpr int D = NBUF - 1;           // LDS ring: D K steps in flight under the MFMAs
    constexpr int A_R64 = A_SLOTS / 64;   // 64-slot DMA rounds of the weight slice
    static_assert(A_SLOTS % 64 == 0 && B_SLOTS % NT == 0, "slot rounds");
    __shared__ __attribute__((aligned(1024))) uint8_t lds[NBUF * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // DMA instructions this wave issues per K step: its weight rounds + the pixel rounds
    const int ops = CPS * ((A_R64 - wave + NWV - 1) / NWV + B_SLOTS / NT);
    const int wp = wave % PW, wc = wave / PW;  // pixel quarter / half, cout half
    // XCD-aware order: the dispatcher deals blockIdx round-robin over the 8 XCDs, so logical
    // blocks (tile, cout block; couts fastest) are renumbered to give every XCD a contiguous
    // range — the cout blocks of a tile then run on one XCD and share its input through that
    // L2 (blockIdx order spread them over n_nb XCDs, each fetching the tile).  A bijection for
    // any grid size: XCD x < r holds q + 1 logical blocks, the others q.
    long lb = blockIdx.x;
    if (p.xcd_order) {
        const long nbk = gridDim.x, q = nbk >> 3, r = nbk & 7, x = blockIdx.x & 7, loc = blockIdx.x >> 3;
        lb = x < r ? x * (q + 1) + loc : r * (q + 1) + (x - r) * q + loc;
    }
    const long tile = lb / p.n_nb;
    const int co0 = (int)(lb - tile * p.n_nb) * BN;
    const long m0 = tile * BMP;
    const int kc = p.cin / 32;            // chunks per tap
    const int nq = KS * KS * kc;          // 32-channel K chunks
    const int K = nq * 32;
    const int nk = (nq + CPS - 1) / CPS;  // ring steps
    // LDS images are row-major with a swizzle: row r (a cout of A, a pixel of B) keeps its
    // four 16-B K chunks (32 channels) in slots 4r .. 4r+3, chunk kg at 4r + (kg ^ swz(r)),
    // swz(r) = -(r >> 2) & 3.  A DMA instruction then reads 16 rows x 64 contiguous bytes
    // (4 lanes per row) instead of 64 rows x 16 B: a quarter of the cache lines per
    // instruction.  The swizzle keeps the 16-lane fragment reads (16 rows, one chunk)
    // conflict-free in every ds_read_b128 lane group.
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    constexpr int BR = B_SLOTS / NT;  // pixel rounds per thread (FP / 2)
    long bm[BR];
    bool bvalid[BR];
    int bkg[BR], bn_[BR], bho[BR], bwo[BR];
#pragma unroll
    for (int j = 0; j < BR; j++) {
        const int slot = j * NT + tid, row = slot >> 2;
        bkg[j] = (slot & 3) ^ swz(row);
        bm[j] = m0 + row;
        bvalid[j] = bm[j] < p.M;
        bn_[j] = bho[j] = bwo[j] = 0;
        if (KS > 1 && bvalid[j]) {
            const long hw = (long)p.Ho * p.Wo;
            bn_[j] = (int)(bm[j] / hw);
            const int r = (int)(bm[j] - (long)bn_[j] * hw);
            bho[j] = r / p.Wo;
            bwo[j] = r - bho[j] * p.Wo;
        }
    }
    // per-thread DMA sources fixed for the launch: the weight rows of this wave's rounds
    // (advanced by 32 channels per K step), and each pixel's image base (the tap moves it)
    constexpr int ARW = (A_R64 + NWV - 1) / NWV;
    const uint16_t* asrc[ARW];
    const int wstep = p.wimg ? p.npad * 32 : 32;  // elements between K steps of a weight row
#pragma unroll
    for (int j = 0; j < ARW; j++) {
        const int sl = (wave + j * NWV) * 64 + lane;
        const int co = sl >> 2, kg = (sl & 3) ^ swz(co);
        asrc[j] = (co0 + co >= p.npad) ? nullptr
                  : p.wimg             ? p.wimg + ((size_t)co0 * 4 + sl) * 8
                                       : p.w + (size_t)(co0 + co) * K + kg * 8;
    }
    const uint16_t* bimg[BR];
#pragma unroll
    for (int j = 0; j < BR; j++) bimg[j] = p.x + (size_t)bn_[j] * p.H * p.W * p.xs;
    int it_ch = 0, it_kh = 0, it_kw = 0;  // (tap, chunk) of the next issued K step (issued in order)
    // one 32-channel chunk q into sub-slot `base`; chunks past the end DMA zeros (every step
    // issues the same number of operations, which the vmcnt accounting relies on)
    auto issue_chunk = [&](int q, uint8_t* base) {
        const bool live = q < nq;
        const int k0 = q * 32;
#pragma unroll
        for (int j = 0; j < ARW; j++) {
            const int r = wave + j * NWV;
            if (r < A_R64) {  // wave-uniform
                const void* src = (live && asrc[j]) ? (const void*)(asrc[j] + (size_t)q * wstep)
                                                    : (const void*)(p.zero + ((r * 64 + lane) & 1023) * 8);
                glds16_det(src, base + r * 64 * 16);
            }
        }
        int hoff = 0, woff = 0, coff = 0;
        if (KS > 1) {
            hoff = it_kh - PAD, woff = it_kw - PAD, coff = it_ch * 32;
            if (live && ++it_ch == kc) {
                it_ch = 0;
                if (++it_kw == KS) it_kw = 0, it_kh++;
            }
        }
#pragma unroll
        for (int j = 0; j < BR; j++) {
            const uint16_t* px = nullptr;
            if (KS == 1) {
                if (bvalid[j] && live) px = p.x + bm[j] * p.xs + k0;
            } else if (live) {
                const int hi = bho[j] * S + hoff, wi = bwo[j] * S + woff;
                if (bvalid[j] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
                    px = bimg[j] + ((size_t)hi * p.W + wi) * p.xs + coff;
            }
            const void* src = px ? (const void*)(px + bkg[j] * 8)
                                 : (const void*)(p.zero + ((j * NT + tid) & 1023) * 8);
            glds16_det(src, base + (A_SLOTS + j * NT + wave * 64) * 16);
        }
    };
    auto issue = [&](int k, int buf) {
#pragma unroll
        for (int c = 0; c < CPS; c++) issue_chunk(k * CPS + c, lds + buf * STAGE + c * SUB);
    };
    f32x4 acc[FP][WCT];
#pragma unroll
    for (int i = 0; i < FP; i++)
#pragma unroll
        for (int c = 0; c < WCT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < D && j < nk; j++) issue(j, j);
    wait_vm(ops * (min(D, nk) - 1));  // step 0 landed, the others in flight
    __builtin_amdgcn_s_barrier();
    const int kg = lane >> 4, r16 = lane & 15;
    const int soff = r16 * 64 + ((kg ^ ((-(r16 >> 2)) & 3)) * 16);  // this lane's (row, chunk) in a 16-row block
    int buf = 0;
    for (int k = 0; k < nk; k++) {
        // ring slot (k + D) % NBUF was last read in step k - 1, which every wave has finished
        if (k + D < nk) issue(k + D, buf == 0 ? NBUF - 1 : buf - 1);
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) {
            const uint8_t* base = lds + buf * STAGE + cc * SUB;
            bf16x8 a[WCT], b[FP];
#pragma unroll
            for (int c = 0; c < WCT; c++)
                a[c] = *reinterpret_cast<const bf16x8*>(base + (wc * (BN / 2) + c * 16) * 64 + soff);
#pragma unroll
            for (int i = 0; i < FP; i++)
                b[i] = *reinterpret_cast<const bf16x8*>(base + A_SLOTS * 16 + (wp * 16 * FP + i * 16) * 64 + soff);
#pragma unroll
            for (int i = 0; i < FP; i++)
#pragma unroll
                for (int c = 0; c < WCT; c++)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[i], acc[i][c], 0, 0, 0);
        }
        // step k + 1 must have landed; the steps issued after it may stay in flight.  A plain
        // s_barrier (no release fence: __syncthreads would drain every DMA in flight)
        wait_vm(ops * max(0, min(k + D, nk - 1) - k - 1));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        buf = buf == NBUF - 1 ? 0 : buf + 1;
    }
    // epilogue: lane holds couts (lane >> 4) * 4 + j of pixel (lane & 15) in each tile
#pragma unroll
    for (int c = 0; c < WCT; c++) {
        const int co = co0 + wc * (BN / 2) + c * 16 + kg * 4;
        if (co >= p.N) continue;
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
#pragma unroll
        for (int i = 0; i < FP; i++) {
            const long m = m0 + wp * 16 * FP + i * 16 + r16;
            if (m >= p.M) continue;
            float v[4] = {acc[i][c][0] + bb.x, acc[i][c][1] + bb.y, acc[i][c][2] + bb.z, acc[i][c][3] + bb.w};
            if (p.act == 2)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = act_f(v[e], 2);
            if (p.res) {
                const uint2 r = *reinterpret_cast<const uint2*>(p.res + m * p.rs + co);
                v[0] += bf(r.x & 0xffff), v[1] += bf(r.x >> 16), v[2] += bf(r.y & 0xffff), v[3] += bf(r.y >> 16);
            }
            if (p.act == 1)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
            *reinterpret_cast<uint2*>(p.y + m * p.ys + co) =
                uint2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)};
        }
    }
}

constexpr int kPersMaxN = 1024;  // couts whose biases the persistent 1x1 kernel stages in LDS

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    typedef __attribute__((address_space(3))) const uint8_t lds_u8;
    return (uint32_t)(uintptr_t)(lds_u8*)p;
}
// LDS write / read-back of the epilogue staging as asm: the compiler would otherwise put a
// vmcnt(0) (the in-flight ring DMAs) in front of them; the read waits for the wave's writes
__device__ __forceinline__ void lds_write_u2(void* p, uint2 v) {
    asm volatile("ds_write_b64 %0, %1\n\ts_nop 1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
// raw buffer resource (stride 0, num_records bytes; gfx9 dword 3)
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    return i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)),
                 __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}
// a weight-fragment load the compiler does not see (its waitcnt pass, seeing the LDS-DMAs and these
// loads as mixed event kinds, put vmcnt(0) in front of every third K step's MFMAs); the kernel's
// own end-of-step wait covers it
__device__ __forceinline__ bf16x8 buffer_load_frag(i32x4 r, int off) {
#ifdef PERS_BUILTIN_LOAD
    __amdgpu_buffer_rsrc_t rr;
    __builtin_memcpy(&rr, &r, 16);
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
#else
    bf16x8 v;
    // s_nop 4: the descriptor may be fresh from v_readfirstlane and the offset from a VALU op
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
#endif
}
// a buffer store the compiler does not see: its waitcnt pass would otherwise count it among the
// pending vector-memory events, see reads and writes mixed, and put vmcnt(0) in front of the next
// use of any load (the weight fragments two K steps ahead); the kernel's own waits count loads only
__device__ __forceinline__ void buffer_store_u4(u32x4 v, i32x4 r, int off) {
#ifdef PERS_BUILTIN_STORE
    __amdgpu_buffer_rsrc_t rr;
    __builtin_memcpy(&rr, &r, 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, rr, off, 0, 0);
#else
    // s_nop 4 as the load; s_nop 1 after: the store reads its data registers late, and the
    // compiler's next instruction may overwrite them
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" : : "v"(v), "v"(off), "s"(r) : "memory");
#endif
}
// this thread's two landed pixel chunks (16 B each) and their 4 scale quads in one wait (early
// clobber: a result register must not alias an address the later reads still need)
__device__ __forceinline__ void lds_read_ca6(const void* d0, const void* d1, const void* t0, const void* t1, u32x4& v0,
                                             u32x4& v1, f32x4& s00, f32x4& s01, f32x4& s10, f32x4& s11) {
    asm volatile(
        "ds_read_b128 %0, %6\n\tds_read_b128 %1, %7\n\tds_read_b128 %2, %8\n\tds_read_b128 %3, %8 offset:16\n\t"
        "ds_read_b128 %4, %9\n\tds_read_b128 %5, %9 offset:16\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(s00), "=&v"(s01), "=&v"(s10), "=&v"(s11)
        : "v"(lds_addr(d0)), "v"(lds_addr(d1)), "v"(lds_addr(t0)), "v"(lds_addr(t1))
        : "memory");
}
__device__ __forceinline__ void lds_write_u4(void* p, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1\n\ts_nop 1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 lds_read_u4_sync(const void* p) {
    u32x4 v;
    asm volatile("s_waitcnt lgkmcnt(0)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}

// ds_read_b128 + its own lgkmcnt(0) in one asm block: the compiler cannot see it, so it inserts
// no vmcnt wait for the LDS-DMAs in flight (it assumes they may alias any LDS read it emits)
__device__ __forceinline__ float4 lds_read_f4_sync(const float* p) {
    typedef __attribute__((address_space(3))) float lds_float;
    const uint32_t a = (uint32_t)(uintptr_t)(const lds_float*)p;
    float4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// Persistent 1x1 GEMM (round 6).  det_conv_gemm_kernel moves both operands by LDS-DMA; on the
// 1x1 convs (~17 ms of the 512-frame forward) that is ~114 cycles per 1-KiB DMA instruction per
// CU (24.6 GB/s per CU, 6.3 TB/s chip-wide: neck.top_down_blocks.1's main+short conv, 20
// instructions per K step of which 12 are the re-fetched weight slice), the kernels' bound.
// Here the pixel operand (B) still arrives by LDS-DMA into a 3-slot ring, but each wave loads
// its own weight fragments (A) straight into VGPRs with buffer loads (L2-resident, no
// redundancy: PW = 1 puts the 4 waves side by side along the couts, each over all 128 pixels),
// two K steps ahead.  A workgroup per (CU, slot) walks a strided list of (tile, cout block)
// items and the pipeline runs across items.  The epilogue stages each wave's 16-pixel rows in
// LDS and writes whole pixel runs with buffer stores.  Same MFMA operands and sequence (K steps
// 0 .. nq - 1 from zero) and epilogue arithmetic as det_conv_gemm_kernel<BN, 1, 1, ...>:
// bit-identical outputs.
// FM (fold mode): 1 = K channels [0, up_c) read from the nearest-2x upsample's source (the
// neck's DET_UP2 op is not run: the pixel DMA addresses the half-resolution pixel); 2 = the
// channel-attention scale (the DET_CA op's in-place pass is not run): wave 0 DMAs each step's
// table of scales (8 frames x 32 channels, f32) one step ahead, and every thread scales its own
// landed pixel chunks in LDS (f32 product, bf16 round: ca_scale_kernel's arithmetic) before the
// barrier that publishes the step.
template <int B, int E, typename F>
__device__ __forceinline__ void det_static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        det_static_for<B + 1, E>(f);
    }
}

template <int BN, int PW, int NBUF, int KS = 1, int STR = 1, int FM = 0>
__global__ __launch_bounds__(256, 2) void det_conv1x1_pers_kernel(GParams p) {
    constexpr int NT = 256, NWV = 4, BMP = 128, D = NBUF - 1;
    constexpr int CWV = NWV / PW;        // waves along the couts
    constexpr int WCO = BN / CWV;        // couts per wave
    constexpr int WCT = WCO / 16;        // 16-cout tiles per wave
    constexpr int FP = BMP / (16 * PW);  // 16-pixel fragments per wave
    constexpr int B_SLOTS = 4 * BMP, SUB = B_SLOTS * 16, BR = B_SLOTS / NT;
    constexpr int ROWB = WCO * 2;        // staged bytes per pixel
    constexpr int OFF_BIAS = NBUF * SUB, OFF_STAGE = OFF_BIAS + kPersMaxN * 4;
    constexpr int OFF_CA = OFF_STAGE + NWV * 16 * ROWB;  // FM & 2: NBUF 1-KiB scale tables
    static_assert(WCO % 16 == 0 && FP * 16 * PW == BMP && B_SLOTS % NT == 0, "tiling");
    static_assert(KS == 1 || FM == 0, "folds: 1x1 only");
    static_assert(!(FM & 2) || BR == 2, "lds_read_ca6: two chunks per thread");
    // one LDS object: with a second __shared__ array the compiler's LDS-DMA alias check put
    // vmcnt(0) in front of every fragment read
    __shared__ __attribute__((aligned(1024))) uint8_t lds[OFF_CA + ((FM & 2) ? NBUF * 1024 : 0)];
    float* bias_s = reinterpret_cast<float*>(lds + OFF_BIAS);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = wave % PW, wc = wave / PW;
    const int kc = p.cin / 32;        // 32-channel chunks per tap
    const int nq = KS * KS * kc;      // K steps per item: (tap, chunk), chunks fastest
    // items: logical blocks (tile, cout block; couts fastest) split into 8 contiguous XCD ranges
    // (the dispatcher deals blockIdx round-robin over the XCDs); XCD x's gx workgroups take its
    // range round-robin, so the cout blocks of a tile run side by side on one XCD
    const long nblk = (p.M + BMP - 1) / BMP * p.n_nb;
    const int G = gridDim.x, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int gx = G / 8 + (xcd < (G & 7) ? 1 : 0);
    const long qx = nblk >> 3, rx = nblk & 7;
    const long x0 = xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx;
    const long x1 = x0 + qx + (xcd < rx ? 1 : 0);
    const long n_items = x1 - x0 > loc ? (x1 - x0 - loc + gx - 1) / gx : 0;
    const long S = n_items * nq;  // K steps of this workgroup
    if (S == 0) return;           // workgroup-uniform
    for (int i = tid; i < p.N; i += NT) bias_s[i] = p.bias[i];
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    const int kg = lane >> 4, r16 = lane & 15;
    int b_row[BR], b_kg[BR];
#pragma unroll
    for (int j = 0; j < BR; j++) {
        const int slot = j * NT + tid;
        b_row[j] = slot >> 2;
        b_kg[j] = (slot & 3) ^ swz(b_row[j]);
    }
    // A: lane (kg, r16) of tile c holds chunk kg of cout co0 + wc * WCO + 16c + r16 (the packed
    // image's slot (q * npad + co) * 4 + (kg ^ swz(co)))
    const i32x4 wr = make_rsrc(p.wimg, (int)std::min<long>((long)p.npad * nq * 64, 0x7fffffffL));
    const int a_step = p.npad * 64;  // bytes between K steps of the image
    int a_lane[WCT];                 // this lane's byte offset per tile for co0 = 0 (step 0)
#pragma unroll
    for (int c = 0; c < WCT; c++) {
        const int co = wc * WCO + c * 16 + r16;
        a_lane[c] = co * 64 + ((kg ^ swz(co)) * 16);
    }
    bf16x8 areg[NBUF][WCT];
    // issue K step g (item g / nq, step g % nq): its pixel image into ring slot ST, its weight
    // fragments into areg[ST]
    // the issue stream (steps are issued in order): its item, step in the item and, for 3x3, the
    // tap and chunk of that step and the output pixels (frame, row, column) of this thread's B
    // rows -- advanced per step, so no division in the per-step path
    long i_it = 0, i_tile = 0;
    int i_k = 0, i_co0 = 0, i_ch = 0, i_kw = 0, i_kh = 0;
    int b_n[BR], b_ho[BR], b_wo[BR];
    long b_up[BR];  // FM & 1: the half-resolution source pixel of each B row
    const long hw = (long)p.Ho * p.Wo;
    // FM & 2: first frame of the scale table of the next issued step; its DMA (wave 0): lane l
    // holds the scales of channels 4 (l & 7) .. + 3 of the step's 32, frame n0 + (l >> 3)
    long ca_n0 = 0;
    auto ca_table = [&](int slot, long n0, int kk) {
        const long nfr = p.M / hw;
        const long fr = std::min<long>(n0 + (lane >> 3), nfr - 1);
        glds16_det(p.ca + fr * p.cin + kk * 32 + (lane & 7) * 4, lds + OFF_CA + slot * 1024);
    };
    auto issue = [&](auto Ss) {
        constexpr int ST = decltype(Ss)::value;
        if (i_k == 0) {  // a new item
            const long lb = x0 + loc + i_it * gx;
            i_tile = lb / p.n_nb;
            i_co0 = (int)(lb - i_tile * p.n_nb) * BN;
            if constexpr (KS > 1) {
                const long hw = (long)p.Ho * p.Wo;
#pragma unroll
                for (int j = 0; j < BR; j++) {
                    const long m = i_tile * BMP + b_row[j];
                    b_n[j] = m < p.M ? (int)(m / hw) : -1;
                    const int r = m < p.M ? (int)(m - (long)b_n[j] * hw) : 0;
                    b_ho[j] = r / p.Wo;
                    b_wo[j] = r - b_ho[j] * p.Wo;
                }
            }
            if constexpr ((FM & 1) != 0) {
#pragma unroll
                for (int j = 0; j < BR; j++) {
                    const long m = i_tile * BMP + b_row[j];
                    b_up[j] = 0;
                    if (m < p.M) {
                        const long n = m / hw;
                        const int r = (int)(m - n * hw), h = r / p.W, w = r - h * p.W;
                        b_up[j] = (n * (p.H >> 1) + (h >> 1)) * (p.W >> 1) + (w >> 1);
                    }
                }
            }
        }
        const int k = i_k;
        uint8_t* base = lds + ST * SUB;
        if constexpr (KS == 1) {
#pragma unroll
            for (int j = 0; j < BR; j++) {
                const long m = i_tile * BMP + b_row[j];
                const uint16_t* px = p.x + m * p.xs;
                if constexpr ((FM & 1) != 0)
                    if (k * 32 < p.up_c) px = p.up + b_up[j] * p.up_s;
                const void* src = m < p.M ? (const void*)(px + k * 32 + b_kg[j] * 8)
                                          : (const void*)(p.zero + ((j * NT + tid) & 1023) * 8);
                glds16_det(src, base + (j * NT + wave * 64) * 16);
            }
        } else {
            // the GEMM kernel's K order: chunk fastest, then the tap column, then the tap row
#pragma unroll
            for (int j = 0; j < BR; j++) {
                const int hi = b_ho[j] * STR + i_kh - KS / 2, wi = b_wo[j] * STR + i_kw - KS / 2;
                const bool in = b_n[j] >= 0 && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
                const void* src = in ? (const void*)(p.x + (((long)b_n[j] * p.H + hi) * p.W + wi) * p.xs + i_ch * 32 + b_kg[j] * 8)
                                     : (const void*)(p.zero + ((j * NT + tid) & 1023) * 8);
                glds16_det(src, base + (j * NT + wave * 64) * 16);
            }
            if (++i_ch == kc) {
                i_ch = 0;
                if (++i_kw == KS) i_kw = 0, i_kh++;
            }
        }
#pragma unroll
        for (int c = 0; c < WCT; c++) {
            // couts past npad: an out-of-range offset (the load returns zeros)
            const int off = i_co0 + wc * WCO + c * 16 < p.npad ? k * a_step + i_co0 * 64 + a_lane[c] : 0x7ff00000;
            areg[ST][c] = buffer_load_frag(wr, off);
        }
        if (++i_k == nq) i_k = 0, i_it++, i_kh = 0;
        if constexpr ((FM & 2) != 0) {  // the next step's scale table (wave 0; clamped past the end)
            if (i_k == 0) ca_n0 = (x0 + loc + i_it * gx) / p.n_nb * BMP / hw;
            if (wave == 0) ca_table((ST + 1) % NBUF, ca_n0, i_k);
        }
    };
    // vector memory instructions per issued step (this wave)
    const int OPS = BR + WCT + ((FM & 2) != 0 && wave == 0 ? 1 : 0);
    // FM & 2: scale this thread's two landed chunks of the step in ring slot `slot` (its own
    // DMAs; the step's table landed one barrier earlier), in the consumption order of the steps
    int sc_k = 0, sc_fs[BR];
    long sc_it = 0;
    auto ca_scale = [&](int slot) {
        if (sc_k == 0) {
            const long tile = (x0 + loc + sc_it * gx) / p.n_nb;
            const long n0 = tile * BMP / hw;
#pragma unroll
            for (int j = 0; j < BR; j++) {
                const long m = tile * BMP + b_row[j];
                sc_fs[j] = m < p.M ? (int)(m / hw - n0) : 0;
            }
        }
        uint8_t* d0 = lds + slot * SUB + tid * 16;
        uint8_t* d1 = d0 + NT * 16;
        const uint8_t* tb = lds + OFF_CA + slot * 1024;
        u32x4 v[2];
        f32x4 sc[2][2];
        lds_read_ca6(d0, d1, tb + sc_fs[0] * 128 + b_kg[0] * 32, tb + sc_fs[1] * 128 + b_kg[1] * 32, v[0], v[1],
                     sc[0][0], sc[0][1], sc[1][0], sc[1][1]);
#pragma unroll
        for (int j = 0; j < 2; j++) {
            float f[8];
            unpack8(uint4{v[j][0], v[j][1], v[j][2], v[j][3]}, f);
#pragma unroll
            for (int e = 0; e < 4; e++) f[e] *= sc[j][0][e], f[4 + e] *= sc[j][1][e];
            const uint4 o = pack8(f);
            lds_write_u4(j ? d1 : d0, u32x4{o.x, o.y, o.z, o.w});
        }
        if (++sc_k == nq) sc_k = 0, sc_it++;
    };
    f32x4 acc[FP][WCT];
#pragma unroll
    for (int i = 0; i < FP; i++)
#pragma unroll
        for (int c = 0; c < WCT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr ((FM & 2) != 0) {  // step 0's scale table, published before the first issue
        ca_n0 = (x0 + loc) / p.n_nb * BMP / hw;
        if (wave == 0) ca_table(0, ca_n0, 0);
        wait_vm(0);
        __builtin_amdgcn_s_barrier();
    }
    det_static_for<0, D>([&](auto J) {
        if (J < S) issue(J);
    });
    wait_vm(OPS * (int)(std::min<long>(D, S) - 1));
    if constexpr ((FM & 2) != 0) {
        ca_scale(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const int soff = r16 * 64 + ((kg ^ ((-(r16 >> 2)) & 3)) * 16);
    uint8_t* stage = lds + OFF_STAGE + wave * 16 * ROWB;  // this wave's epilogue rows
    int k = 0;
    long it = 0;
    unsigned ends = 0;  // bit t: iteration g - 1 - t ran an epilogue
    constexpr int kStores = FP * ((2 * WCO + 63) / 64);  // store instructions per epilogue (this wave)
    auto step = [&](long g, auto Ss) {
        constexpr int ST = decltype(Ss)::value;
        if (g + D < S) issue(std::integral_constant<int, (ST + D) % NBUF>{});
        {
            // this step's weight fragments landed at the previous step's wait (the asm loads are
            // invisible to the compiler): tell it so here, before their first use
#pragma unroll
            for (int c = 0; c < WCT; c++) asm volatile("" : "+v"(areg[ST][c]));
            const uint8_t* base = lds + ST * SUB;
            bf16x8 b[FP];
#pragma unroll
            for (int i = 0; i < FP; i++) b[i] = *reinterpret_cast<const bf16x8*>(base + (wp * 16 * FP + i * 16) * 64 + soff);
#pragma unroll
            for (int i = 0; i < FP; i++)
#pragma unroll
                for (int c = 0; c < WCT; c++)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(areg[ST][c], b[i], acc[i][c], 0, 0, 0);
        }
        // step g + 1 landed (pixels and weights): younger are the later steps' operations and
        // the stores of the epilogues run since its issue (iterations g + 1 - D .. g - 1).  Loads,
        // stores and LDS-DMA retire in issue order, so counting the stores keeps their slow write
        // acknowledgements off this wait.
        wait_vm(OPS * (int)(std::min<long>(g + D, S - 1) - g - 1) + kStores * __builtin_popcount(ends & ((1u << (D - 1)) - 1)));
        ends <<= 1;
        if constexpr ((FM & 2) != 0)
            if (g + 1 < S) ca_scale((ST + 1) % NBUF);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (++k < nq) return;
        // ---- the item's epilogue (det_conv_gemm_kernel's arithmetic), a fresh accumulator
        const long lb = x0 + loc + it * gx;
        const long tile = lb / p.n_nb;
        const int co0 = (int)(lb - tile * p.n_nb) * BN;
        const long m0 = tile * BMP;
        float4 bb[WCT];
#pragma unroll
        for (int c = 0; c < WCT; c++) {
            const int co = co0 + wc * WCO + c * 16 + kg * 4;
            bb[c] = lds_read_f4_sync(bias_s + (co < p.N ? co : 0));
        }
        // buffer stores: lanes past the couts / pixels get an out-of-range offset and are dropped
        const long mv = p.M - m0;
        const i32x4 yr = make_rsrc(p.y + m0 * p.ys, (int)((mv < BMP ? mv : BMP) * p.ys * 2));
#pragma unroll
        for (int i = 0; i < FP; i++) {
            const long mi = m0 + wp * 16 * FP + i * 16;
#pragma unroll
            for (int c = 0; c < WCT; c++) {
                const int co = co0 + wc * WCO + c * 16 + kg * 4;
                const long m = mi + r16;
                float v[4] = {acc[i][c][0] + bb[c].x, acc[i][c][1] + bb[c].y, acc[i][c][2] + bb[c].z,
                              acc[i][c][3] + bb[c].w};
                acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (p.act == 2)
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = act_f(v[e], 2);
                if (p.res && co < p.N && m < p.M) {
                    const uint2 r = *reinterpret_cast<const uint2*>(p.res + m * p.rs + co);
                    v[0] += bf(r.x & 0xffff), v[1] += bf(r.x >> 16), v[2] += bf(r.y & 0xffff), v[3] += bf(r.y >> 16);
                }
                if (p.act == 1)
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
                lds_write_u2(stage + r16 * ROWB + (c * 16 + kg * 4) * 2,
                             uint2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)});
            }
            // the wave's 16 pixels x WCO couts back as 16-B row chunks: a store instruction writes
            // whole ROWB-byte pixel runs instead of 16 runs of 32 B
            constexpr int NCH = 16 * ROWB / 16;
#pragma unroll
            for (int q0 = 0; q0 < NCH; q0 += 64) {
                const int q = min(q0 + lane, NCH - 1);
                const int px = q / (ROWB / 16), ch = q - px * (ROWB / 16);
                const u32x4 o = lds_read_u4_sync(stage + q * 16);
                const int co = co0 + wc * WCO + ch * 8;
                const bool ok = q0 + lane < NCH && co < p.N;
                const int off = ok ? ((wp * 16 * FP + i * 16 + px) * p.ys + co) * 2 : 0x7ff00000;
                buffer_store_u4(o, yr, off);
            }
        }
        ends |= 1;
        k = 0;
        it++;
    };
    for (long g = 0; g < S; g += NBUF)
        det_static_for<0, NBUF>([&](auto J) {
            if (g + J < S) step(g + J, J);
        });
}

// 3x3/s1 convs with one 32-channel input chunk (the 320x320 stem / stage-1 planes, 24 -> 32
// padded channels): im2col re-DMAs every input pixel once per tap while a tap's K work is a
// single chunk, so the GEMM kernel above is DMA-issue bound there.  Here a tile is 2 output
// rows x 64 columns of one frame; its 4 x 66 input halo (64 B per pixel) and all 9 taps'
// weights arrive in one DMA phase, and the taps are LDS offsets.  Same swizzled row-major
// images as the GEMM kernel (row = halo pixel / cout, 4 16-B chunks per row); the
// workgroup then runs its 9 K-steps without another barrier (3 workgroups per CU hide the
// DMA).  One chunk: K order (tap, channel) as the GEMM kernel, identical sums; two chunks
// (64 channels, one DMA + compute phase each): chunk-major K order, equal to f32 rounding.
// TR output rows per tile (2 or 4): wave (wp, wc) computes rows wp, wp + 2, ... of cout half
// wc.  4 rows spread each tile's weight DMA over twice the pixels (62.5 KB of LDS, 2
// workgroups per CU, against 54 KB and 3 for 2 rows); the K order per output is the same.
// LT > 0 (round 6): only the first LT 16-cout tiles carry real channels (RTMDet-m's 48-channel
// stem / stage-1 convs stored as 64: the last tile's weights and biases are zero, so its outputs
// are SiLU(0) = +0).  Each of the 4 waves then takes one output row of a 4-row tile and all LT
// tiles (12 MFMAs per tap instead of 16: the zero tile is not multiplied) and stores zeros for
// the padding couts — the real couts' K order and epilogue are unchanged: bit-identical.
template <int BN, int NCK, int TR = 2, int LT = 0>  // NCK 32-channel input chunks, one DMA + compute phase each
__global__ __launch_bounds__(256, TR == 2 ? 3 : 2) void det_conv_halo_kernel(GParams p) {
    constexpr bool ROWS = LT > 0;
    static_assert(!ROWS || (TR % 4 == 0 && LT < BN / 16), "live-tile halo: 4-row tiles");
    constexpr int TW = 64, HW_ = TW + 2, HP = (TR + 2) * HW_;  // halo pixels
    constexpr int RS = ROWS ? 4 : 2;                           // row stride between a wave's rows
    constexpr int NRW = TR / RS;                               // output rows per wave
    constexpr int A_SLOTS = 9 * 4 * BN, A_R64 = A_SLOTS / 64;
    constexpr int B_R64 = (HP * 4 + 63) / 64;
    constexpr int WCT = ROWS ? LT : BN / 32;                   // 16-cout tiles per wave
    __shared__ __attribute__((aligned(1024))) uint8_t lds[(A_SLOTS + B_R64 * 64) * 16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = ROWS ? wave : wave & 1, wc = ROWS ? 0 : wave >> 1;  // output row of the tile, cout half
    const int tiles_w = (p.W + TW - 1) / TW, tiles_h = (p.H + TR - 1) / TR;
    const int per = tiles_w * tiles_h;
    const int n = blockIdx.x / per, t = blockIdx.x - n * per;
    const int ho0 = (t / tiles_w) * TR, wo0 = (t - (t / tiles_w) * tiles_w) * TW;
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    const uint16_t* xb = p.x + (size_t)n * p.H * p.W * p.xs;
    const int kg = lane >> 4, r16 = lane & 15;
    const int soff = r16 * 64 + ((kg ^ swz(r16)) * 16);
    f32x4 acc[NRW][4][WCT];
#pragma unroll
    for (int rw = 0; rw < NRW; rw++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < WCT; c++) acc[rw][i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < NCK; q++) {
    if (q > 0) __builtin_amdgcn_s_barrier();  // every wave is done with chunk q-1's images
    // weights: slot s of tap tp = tp * 4BN + 4co + (kg ^ swz(co))
    for (int r = wave; r < A_R64; r += 4) {
        const int sl = r * 64 + lane, tp = sl / (4 * BN), rem = sl - tp * (4 * BN);
        const int co = rem >> 2, kq = (rem & 3) ^ swz(co);
        glds16_det(p.w + (size_t)co * (288 * NCK) + tp * (32 * NCK) + q * 32 + kq * 8, lds + r * 64 * 16);
    }
    // input halo: slot s = 4hp + (kg ^ swz(hp)), hp = halo row * 66 + halo col
    for (int r = wave; r < B_R64; r += 4) {
        const int sl = r * 64 + lane, hp = sl >> 2, kq = (sl & 3) ^ swz(hp);
        const int hy = hp / HW_, hx = hp - hy * HW_;
        const int gy = ho0 + hy - 1, gx = wo0 + hx - 1;
        const bool in = hp < HP && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
        const void* src = in ? (const void*)(xb + ((size_t)gy * p.W + gx) * p.xs + q * 32 + kq * 8)
                             : (const void*)(p.zero + (sl & 1023) * 8);
        glds16_det(src, lds + (A_SLOTS + r * 64) * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int tp = 0; tp < 9; tp++) {
        const int dy = tp / 3, dx = tp % 3;
        bf16x8 a[WCT], b[NRW][4];
#pragma unroll
        for (int c = 0; c < WCT; c++)
            a[c] = *reinterpret_cast<const bf16x8*>(lds + tp * 4 * BN * 16 + (wc * (BN / 2) + c * 16) * 64 + soff);
#pragma unroll
        for (int rw = 0; rw < NRW; rw++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int hp = (wp + RS * rw + dy) * HW_ + i * 16 + r16 + dx;
                b[rw][i] = *reinterpret_cast<const bf16x8*>(lds + A_SLOTS * 16 + hp * 64 + ((kg ^ swz(hp)) * 16));
            }
#pragma unroll
        for (int rw = 0; rw < NRW; rw++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < WCT; c++)
                    acc[rw][i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[rw][i], acc[rw][i][c], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int rw = 0; rw < NRW; rw++) {
    const int ho = ho0 + wp + RS * rw;
    if (ho >= p.H) break;
    if constexpr (ROWS) {   // the zero tiles' couts
#pragma unroll
        for (int c = LT; c < BN / 16; c++) {
            const int co = c * 16 + kg * 4;
            if (co >= p.N) continue;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int wo = wo0 + i * 16 + r16;
                if (wo >= p.W) continue;
                *reinterpret_cast<uint2*>(p.y + (((long)n * p.H + ho) * p.W + wo) * p.ys + co) = uint2{0u, 0u};
            }
        }
    }
#pragma unroll
    for (int c = 0; c < WCT; c++) {
        const int co = wc * (BN / 2) + c * 16 + kg * 4;
        if (co >= p.N) continue;
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int wo = wo0 + i * 16 + r16;
            if (wo >= p.W) continue;
            const long m = ((long)n * p.H + ho) * p.W + wo;
            const f32x4 ac = acc[rw][i][c];
            float v[4] = {ac[0] + bb.x, ac[1] + bb.y, ac[2] + bb.z, ac[3] + bb.w};
            if (p.act == 2)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = act_f(v[e], 2);
            if (p.res) {
                const uint2 r = *reinterpret_cast<const uint2*>(p.res + m * p.rs + co);
                v[0] += bf(r.x & 0xffff), v[1] += bf(r.x >> 16), v[2] += bf(r.y & 0xffff), v[3] += bf(r.y >> 16);
            }
            if (p.act == 1)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
            *reinterpret_cast<uint2*>(p.y + m * p.ys + co) =
                uint2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)};
        }
    }
    }
}

// Persistent halo conv (round 6) for the 64-cout 3x3/s1 convs with one or two input chunks (the
// 320x320 stem.2 and the 160x160 stage-1 block conv1s: ~6.6 ms of the 512-frame forward).
// det_conv_halo_kernel re-DMAs the conv's whole weight set (36 KB per chunk) with every
// 256-pixel tile: 60 % of its LDS-DMA bytes, and without them the forward ran 3.2 ms faster
// (timing diagnostic, profiles/r06_det_halo_pers.txt).  Here one workgroup per CU (8 waves)
// keeps the weights of every chunk resident in LDS for the launch and walks 8-row x 64-column
// tiles (a contiguous per-XCD range, so neighbouring tiles' halo rows meet in that L2); each
// (tile, chunk) step's 10 x 66 halo arrives by LDS-DMA into one of two buffers while the
// previous step computes.  Wave w computes output row w of the tile for the LT live 16-cout
// tiles (4 pixel fragments each); the padding couts are stored as zeros (their weights and
// biases are zero).  The DMA and the stores are asm the compiler does not track (no vmcnt it
// would put in front of LDS reads); the kernel counts its own waits.  Same operand images and
// K order (chunk, tap, channel) as det_conv_halo_kernel: bit-identical.
__device__ __forceinline__ void glds16_raw(const void* src, uint32_t lds_off) {
    uint32_t saved;  // m0 is the compiler's: restored after the issue (the DMA reads it at issue)
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "v"(src), "s"(lds_off)
                 : "memory");
}
__device__ __forceinline__ void buffer_store_u2v(u32x2 v, i32x4 r, int off) {
    asm volatile("s_nop 4\n\tbuffer_store_dwordx2 %0, %1, %2, 0 offen\n\ts_nop 1" : : "v"(v), "v"(off), "s"(r) : "memory");
}

template <int BN_, int NCK, int LT>
struct HaloPersCfg {
    static constexpr int BN = BN_, TR = 8, TW = 64, HW_ = TW + 2, HP = (TR + 2) * HW_;
    static constexpr int NWV = 8, NT = 64 * NWV;
    static constexpr int A_SLOTS = 9 * 4 * BN;              // one chunk's weights, [tap][cout][4]
    static constexpr int B_R64 = (HP * 4 + 63) / 64;        // halo DMA rounds (1 KiB each)
    static constexpr int BUF = B_R64 * 64 * 16;             // one halo buffer
    static constexpr int OFF_B = NCK * A_SLOTS * 16;
    static constexpr int LDS = OFF_B + 2 * BUF;
    static_assert(LDS <= 160 * 1024, "halo pers: LDS budget");
    static_assert(LT >= 1 && LT <= BN / 16 && (BN == 32 || BN == 64), "live tiles");
};

template <int BN_, int NCK, int LT>
__global__ __launch_bounds__(512, 1) void det_conv_halo_pers_kernel(GParams p) {
    using G = HaloPersCfg<BN_, NCK, LT>;
    constexpr int BN = G::BN, TR = G::TR, TW = G::TW, HW_ = G::HW_, NWV = G::NWV;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    const int tiles_w = (p.W + TW - 1) / TW, tiles_h = (p.H + TR - 1) / TR, per = tiles_w * tiles_h;
    const long T = p.M / ((long)p.H * p.W) * per;
    const int NG = gridDim.x, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int gx = NG / 8 + (xcd < (NG & 7) ? 1 : 0);
    const long qx = T >> 3, rx = T & 7;
    const long x0 = xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx;
    const long x1 = x0 + qx + (xcd < rx ? 1 : 0);
    const long n_tiles = x1 - x0 > loc ? (x1 - x0 - loc + gx - 1) / gx : 0;
    if (n_tiles == 0) return;  // workgroup-uniform
    const long S = n_tiles * NCK;
    // the weights of every chunk, once: slot s of chunk q = tap * 4BN + 4co + (kq ^ swz(co))
    for (int i = tid; i < NCK * G::A_SLOTS; i += G::NT) {
        const int q = i / G::A_SLOTS, sl = i - q * G::A_SLOTS, tp = sl / (4 * BN), rem = sl - tp * (4 * BN);
        const int co = rem >> 2, kq = (rem & 3) ^ swz(co);
        *reinterpret_cast<uint4*>(lds + i * 16) =
            *reinterpret_cast<const uint4*>(p.w + (size_t)co * (288 * NCK) + tp * (32 * NCK) + q * 32 + kq * 8);
    }
    const int kg = lane >> 4, r16 = lane & 15;
    // the lane's biases, complete before the loop (a load the compiler still counted as pending
    // there would put a vmcnt wait, covering the next step's DMA, into every epilogue)
    f32x4 bb[LT];
#pragma unroll
    for (int c = 0; c < LT; c++) {
        bb[c] = *reinterpret_cast<const f32x4*>(p.bias + c * 16 + kg * 4);
        asm volatile("" : "+v"(bb[c]));
    }
    auto tile_of = [&](long t, int& n, int& ho0, int& wo0) {
        const long lt = x0 + loc + t * gx;
        n = (int)(lt / per);
        const int r = (int)(lt - (long)n * per), th = r / tiles_w;
        ho0 = th * TR;
        wo0 = (r - th * tiles_w) * TW;
    };
    auto issue = [&](long st, int buf) {
        const long t = st / NCK;
        const int q = (int)(st - t * NCK);
        int n, ho0, wo0;
        tile_of(t, n, ho0, wo0);
        const uint16_t* xb = p.x + (size_t)n * p.H * p.W * p.xs;
#pragma unroll
        for (int j = 0; j < (G::B_R64 + NWV - 1) / NWV; j++) {
            const int r = wave + NWV * j;
            if (r < G::B_R64) {  // wave-uniform
                const int sl = r * 64 + lane, hp = sl >> 2, kq = (sl & 3) ^ swz(hp);
                const int hy = hp / HW_, hx = hp - hy * HW_;
                const int gy = ho0 + hy - 1, gx2 = wo0 + hx - 1;
                const bool in = hp < G::HP && (unsigned)gy < (unsigned)p.H && (unsigned)gx2 < (unsigned)p.W;
                const void* src = in ? (const void*)(xb + ((size_t)gy * p.W + gx2) * p.xs + q * 32 + kq * 8)
                                     : (const void*)(p.zero + (sl & 1023) * 8);
                glds16_raw(src, (uint32_t)(G::OFF_B + buf * G::BUF + r * 1024));
            }
        }
    };
    constexpr int kStores = 4 * (BN / 16);  // per wave and tile: 4 fragments x every 16-cout tile
    const int soff = r16 * 64 + ((kg ^ swz(r16)) * 16);
    f32x4 acc[4][LT];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int c = 0; c < LT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue(0, 0);
    __syncthreads();  // the weights (plain stores) are visible
    int st_after = 0;  // store instructions issued since the last DMA issue
    for (long st = 0; st < S; st++) {
        const int buf = (int)(st & 1);
        wait_vm(st_after);  // this wave's DMA of step st landed (only the later stores may be pending)
        __builtin_amdgcn_s_barrier();  // every wave's; the other buffer is free
        asm volatile("" ::: "memory");
        if (st + 1 < S) {
            issue(st + 1, buf ^ 1);
            st_after = 0;
        }
        const long t = st / NCK;
        const int q = (int)(st - t * NCK);
        const uint8_t* wa = lds + q * G::A_SLOTS * 16;
        const uint8_t* hb = lds + G::OFF_B + buf * G::BUF;
#pragma unroll
        for (int tp = 0; tp < 9; tp++) {
            const int dy = tp / 3, dx = tp % 3;
            bf16x8 a[LT], b[4];
#pragma unroll
            for (int c = 0; c < LT; c++) a[c] = *reinterpret_cast<const bf16x8*>(wa + tp * 4 * BN * 16 + (c * 16) * 64 + soff);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int hp = (wave + dy) * HW_ + i * 16 + r16 + dx;
                b[i] = *reinterpret_cast<const bf16x8*>(hb + hp * 64 + ((kg ^ swz(hp)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < LT; c++) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[i], acc[i][c], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (q + 1 < NCK) continue;
        // ---- the tile's epilogue: row `wave` of the tile, every 16-cout tile (zeros past LT)
        int n, ho0, wo0;
        tile_of(t, n, ho0, wo0);
        const int ho = ho0 + wave;
        const uint16_t* yb = p.y + (((size_t)n * p.H + (ho < p.H ? ho : 0)) * p.W + wo0) * p.ys;
        const i32x4 yr = make_rsrc(yb, (int)std::min<long>((long)TW * p.ys * 2, 0x7fffffffL));
#pragma unroll
        for (int c = 0; c < BN / 16; c++) {
            const int co = c * 16 + kg * 4;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int wo = wo0 + i * 16 + r16;
                u32x2 o = {0u, 0u};
                if (c < LT) {
                    const f32x4 ac = acc[i][c < LT ? c : 0];
                    const f32x4 bc = bb[c < LT ? c : 0];
                    float v[4] = {ac[0] + bc[0], ac[1] + bc[1], ac[2] + bc[2], ac[3] + bc[3]};
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = act_f(v[e], p.act);
                    o = u32x2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)};
                }
                const bool ok = ho < p.H && wo < p.W && co < p.N;
                buffer_store_u2v(o, yr, ok ? ((i * 16 + r16) * p.ys + co) * 2 : 0x7ff00000);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < LT; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
        st_after = kStores;
    }
}

// 3x3/s1 convs with >= 3 input chunks on the 80x80 and 40x40 planes (the CSPNeXt stage-3
// blocks, the neck's 40x40 blocks and out_convs, the head's stacked convs: ~18 of the 38.9
// GMAC per frame).  The im2col GEMM above re-DMAs every input pixel once per tap, 20 KB per
// 786 K MAC (39 MAC/B from L2), which bounds it near a quarter of the MFMA peak.  Here a work
// item is a band of TR output rows x the whole width (320 pixels: 4 x 80 or 8 x 40) of one
// frame and 64 couts; per 32-channel input chunk its (TR + 2) x (W + 2) input halo (64 B per
// pixel, zero borders) and the chunk's weights for all 9 taps ([tap][cout][4 chunks], a
// contiguous 36 KB slice of the packed image, det_pack_band_weights) arrive by one round of
// LDS-DMA into one of two buffers while the previous chunk computes (~88 MAC per byte moved),
// and the taps are address offsets into the halo.  4 waves, each 80 output pixels (5
// fragments of 16) x the 64 couts (4 tiles): every A fragment read feeds 5 MFMAs, every B
// fragment 4 (v_mfma_f32_16x16x32_bf16).  Persistent workgroups, one per CU (137 KB of LDS),
// walk their items chunk by chunk with the next step's DMA in flight.  XCD-aware: the
// workgroups of one XCD (blockIdx % 8) form groups of n_nb (couts / 64) that take the same
// band together, one cout block each, so a band's input comes from HBM once into that XCD's
// L2.  Same swizzled row images as the GEMM kernel (a row = cout or halo pixel, its four 16-B
// channel chunks at 4r + (kg ^ swz(r))).  K order (chunk, tap, channel): equal to the GEMM
// kernel's (tap, chunk, channel) sums to f32 rounding.
constexpr int kBandBN = 64;

template <int W, int TR>
struct BandCfg {
    static constexpr int HWD = W + 2, HP = (TR + 2) * HWD;  // halo row pitch, halo pixels
    static constexpr int P = TR * W;                        // output pixels per item
    static constexpr int A_SLOTS = 9 * 4 * kBandBN;         // [tap][cout][4]
    static constexpr int A_R64 = A_SLOTS / 64;
    static constexpr int B_R64 = (HP * 4 + 63) / 64;
    static constexpr int BUF = (A_SLOTS + B_R64 * 64) * 16;
    static constexpr int LDS = 2 * BUF;
    static constexpr int FPW = P / 64;                      // 16-pixel fragments per wave (4 waves)
    static_assert(P == 320 && FPW == 5, "band: 320-pixel items");
    static_assert(LDS <= 160 * 1024, "band: LDS budget");
};

// (Measured and dropped: a plane-major halo — [4 channel chunks][halo pixel] 16-B slots, tap
// offsets as immediates, no swizzle, 16-B DMA pieces — 23.80 vs 23.32 ms per 128-frame forward,
// gpurun_out/detband4: four times the DMA pieces cost more than the address arithmetic saved.)
// NWV waves: 4 (one per SIMD, each 80 pixels x the 64 couts) or 8 (two per SIMD, each 80 pixels
// x 32 couts: more LDS reads, but a second wave to hide each one's waits).
// (Measured and dropped, round 6: the 20x20 planes as whole-frame items of 400 pixels = 5 pixel
// groups x 2 cout groups, 10 waves: 24 % of the MFMA peak against the GEMM kernel's 31 % there —
// the SIMDs hold 3, 3, 2, 2 waves — 5.58 vs 4.47 ms for the 8 convs, profiles/r06_det_folds.txt.)
template <int W, int TR, int NWV>
__global__ __launch_bounds__(64 * NWV, 1) void det_conv_band_kernel(GParams p, const uint16_t* __restrict__ wband) {
    using C = BandCfg<W, TR>;
    constexpr int FP = C::FPW;
    constexpr int CT = 4 * 4 / NWV;  // 16-cout tiles per wave
    static_assert(NWV == 4 || NWV == 8, "band: 4 or 8 waves");
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = wave & 3, wc = wave >> 2;  // pixel group, cout group
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    // item assignment (see above): WG b on XCD b % 8, group g of n_nb consecutive slots
    const int n_nb = p.n_nb, nck = p.cin / 32;
    const int G = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, sl = b >> 3, spx = G >> 3;
    const int ng = spx / n_nb;
    if (sl >= ng * n_nb) return;  // whole workgroup: uniform
    const int nb = sl % n_nb, g = sl / n_nb;
    const int tpi = p.H / TR;  // bands per frame
    const int tiles = (int)(p.M / ((long)p.H * W)) * tpi;
    const int n_items = tiles > (g * 8 + xcd) ? (tiles - (g * 8 + xcd) + ng * 8 - 1) / (ng * 8) : 0;
    if (n_items == 0) return;
    const int steps = n_items * nck;
    auto item_tile = [&](int k) { return (k * ng + g) * 8 + xcd; };
    // DMA of step st (chunk c of item k) into buffer buf, in 9 parts: part j = this wave's
    // weight round j (9 per wave) and halo round j (<= 8 per wave).  The parts are issued one
    // per tap in the middle of the previous step's MFMAs, so their address arithmetic rides in
    // the MFMA shadow; the halo rounds use per-item source offsets (hoff, recomputed when the
    // next step starts a new item: -1 = outside the frame, the zero region).
    constexpr int HR = (C::B_R64 + NWV - 1) / NWV;  // halo rounds per wave (some waves one fewer)
    constexpr int AR = (C::A_R64 + NWV - 1) / NWV;  // weight rounds per wave (some waves one fewer)
    constexpr int NPART = AR > HR ? AR : HR;         // DMA parts per wave and step
    static_assert(NPART <= 9, "band: DMA parts");
    int hoff[HR];
    const uint16_t* xframe = p.x;
    auto set_item = [&](int k) {
        const int t = item_tile(k), n = t / tpi, row0 = (t - n * tpi) * TR;
        xframe = p.x + (size_t)n * p.H * W * p.xs;
#pragma unroll
        for (int j = 0; j < HR; j++) {
            const int s2 = (wave + NWV * j) * 64 + lane, hp = s2 >> 2, kq = (s2 & 3) ^ swz(hp);
            const int hy = hp / C::HWD, hx = hp - hy * C::HWD;
            const int gy = row0 + hy - 1, gx = hx - 1;
            const bool in = hp < C::HP && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)W;
            hoff[j] = in ? (gy * W + gx) * p.xs + kq * 8 : -1;
        }
    };
    auto issue_part = [&](int st, int buf, int j) {
        const int k = st / nck, c = st - k * nck;
        uint8_t* base = lds + buf * C::BUF;
        const int r = wave + NWV * j;
        if (j < AR && r < C::A_R64)
            glds16_det(wband + ((size_t)(nb * nck + c) * C::A_SLOTS + r * 64 + lane) * 8, base + r * 64 * 16);
        if (j < HR && r < C::B_R64) {
            const int s2 = r * 64 + lane;
            const void* src = hoff[j] >= 0 ? (const void*)(xframe + hoff[j] + c * 32)
                                           : (const void*)(p.zero + (s2 & 1023) * 8);
            glds16_det(src, base + (C::A_SLOTS + s2) * 16);
        }
    };
    const int kg = lane >> 4, r16 = lane & 15;
    const int soffA = (r16 * 4 + (kg ^ swz(r16))) * 16;
    int hb[FP];  // halo index of tap (0, 0) for this lane's pixel of each fragment
#pragma unroll
    for (int i = 0; i < FP; i++) {
        const int px = wp * (FP * 16) + i * 16 + r16, pr = px / W, pc = px - pr * W;
        hb[i] = pr * C::HWD + pc;
    }
    f32x4 acc[FP][CT];
    // one chunk's 9 taps from LDS buffer `base`, with the DMA parts of step `nst` in its first
    // taps (nst < 0: none); tap t + 1's fragments are read in the middle of tap t's MFMAs (two
    // register sets).
    auto compute = [&](const uint8_t* base, int nst, int nbuf) {
        bf16x8 fa[2][CT], fbv[2][FP];
        auto load_a = [&](int tp, int sl) {
#pragma unroll
            for (int ct = 0; ct < CT; ct++)
                fa[sl][ct] =
                    *reinterpret_cast<const bf16x8*>(base + (tp * 4 * kBandBN + (wc * CT + ct) * 64) * 16 + soffA);
        };
        auto load_b = [&](int tp, int sl) {
            const int toff = (tp / 3) * C::HWD + (tp % 3);
#pragma unroll
            for (int i = 0; i < FP; i++) {
                const int hp = hb[i] + toff;
                fbv[sl][i] = *reinterpret_cast<const bf16x8*>(base + (C::A_SLOTS + hp * 4 + (kg ^ swz(hp))) * 16);
            }
        };
        load_b(0, 0);
        load_a(0, 0);
        // per tap: 8 MFMAs, then tap t + 1's 9 fragment reads and this tap's DMA part, then the
        // other 12 MFMAs: the compiler's wait before the next tap (it can only wait for every
        // outstanding LDS read while LDS-DMA is in flight) then covers reads 12 MFMAs old
#pragma unroll
        for (int tp = 0; tp < 9; tp++) {
            const int sl = tp & 1;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++)
                    acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sl][ct], fbv[sl][i], acc[i][ct], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (tp + 1 < 9) {
                load_b(tp + 1, sl ^ 1);
                load_a(tp + 1, sl ^ 1);
            }
            // the next step's DMA in the first 5 taps (2 parts each): it lands well before the
            // step's vmcnt wait
            if constexpr (NPART > 5) {  // 2 parts per tap
                if (nst >= 0 && 2 * tp < NPART) issue_part(nst, nbuf, 2 * tp);
                if (nst >= 0 && 2 * tp + 1 < NPART) issue_part(nst, nbuf, 2 * tp + 1);
            } else {
                if (nst >= 0 && tp < NPART) issue_part(nst, nbuf, tp);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 2; i < FP; i++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++)
                    acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sl][ct], fbv[sl][i], acc[i][ct], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    set_item(0);
#pragma unroll
    for (int j = 0; j < NPART; j++) issue_part(0, 0, j);
    int buf = 0, st = 0;
    for (int k = 0; k < n_items; k++) {
#pragma unroll
        for (int i = 0; i < FP; i++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[i][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nck; c++, st++) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of step st (and stores)
            __builtin_amdgcn_s_barrier();                         // every wave's; buffer buf ^ 1 is free
            asm volatile("" ::: "memory");
            const bool more = st + 1 < steps;
            if (more && c + 1 == nck) set_item(k + 1);  // the next step starts item k + 1
            compute(lds + buf * C::BUF, more ? st + 1 : -1, buf ^ 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            buf ^= 1;
        }
        // epilogue of item k: lane holds couts 16 ct + 4 kg + j of its pixel
        const int t = item_tile(k), n = t / tpi, row0 = (t - n * tpi) * TR;
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            const int co = nb * kBandBN + (wc * CT + ct) * 16 + kg * 4;
            if (co >= p.N) continue;
            const float4 bv = *reinterpret_cast<const float4*>(p.bias + co);
#pragma unroll
            for (int i = 0; i < FP; i++) {
                const int px = wp * (FP * 16) + i * 16 + r16, pr = px / W, pc = px - pr * W;
                const long m = ((long)n * p.H + row0 + pr) * W + pc;
                const f32x4 ac = acc[i][ct];
                float v[4] = {ac[0] + bv.x, ac[1] + bv.y, ac[2] + bv.z, ac[3] + bv.w};
                if (p.act == 2)
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = act_f(v[e], 2);
                if (p.res) {
                    const uint2 rr = *reinterpret_cast<const uint2*>(p.res + m * p.rs + co);
                    v[0] += bf(rr.x & 0xffff), v[1] += bf(rr.x >> 16), v[2] += bf(rr.y & 0xffff),
                        v[3] += bf(rr.y >> 16);
                }
                if (p.act == 1)
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
                *reinterpret_cast<uint2*>(p.y + m * p.ys + co) =
                    uint2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)};
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// band weight image: [nb][chunk][tap][cout 64][4 swizzled 16-B chunks] from w [npad][3][3][cin];
// couts past npad (the last block of a 96-cout conv) are zero rows
__global__ __launch_bounds__(256) void det_pack_band_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ img,
                                                          int npad, int cin) {
    const int nck = cin / 32;
    const int rows = (npad + kBandBN - 1) / kBandBN * kBandBN;
    const long n = (long)rows * 9 * cin / 8;  // 16-B slots
    for (long d = blockIdx.x * 256L + threadIdx.x; d < n; d += (long)gridDim.x * 256) {
        const int q = (int)(d & 3);
        const long r = d >> 2;                  // (nb, chunk, tap, co)
        const int co = (int)(r % kBandBN);
        const long r2 = r / kBandBN;
        const int tp = (int)(r2 % 9);
        const long r3 = r2 / 9;
        const int c = (int)(r3 % nck), nb = (int)(r3 / nck);
        const int kg = q ^ ((-(co >> 2)) & 3);
        const int row = nb * kBandBN + co;
        *reinterpret_cast<uint4*>(img + d * 8) =
            row < npad ? *reinterpret_cast<const uint4*>(w + ((size_t)row * 9 + tp) * cin + c * 32 + kg * 8)
                       : uint4{0u, 0u, 0u, 0u};
    }
}

// ------------------------------------------------------------------ channel attention
// Channel means: kCaSplit workgroups per image each sum a contiguous pixel range (f32
// per-thread partial sums, then an LDS tree) into part[n][split][C]; then one workgroup per
// image adds the splits in order (deterministic), divides by H*W and applies
// s = hardsigmoid(W.mean + b) with W^T [C][C] read coalesced.
constexpr int kCaSplit = 16;

struct CaParams {
    const uint16_t* x;
    const float* wt;  // W^T [k][c]
    const float* b;
    float* part;  // [n][kCaSplit][C]
    float* s;     // [n][C]
    int HW, C, xs;
};

__global__ __launch_bounds__(256) void ca_pool_kernel(CaParams p) {
    extern __shared__ float red[];  // [rows][C]
    const int n = blockIdx.y, sp = blockIdx.x, tid = threadIdx.x;
    const int Q = p.C / 8;
    const int rows = 256 / Q;  // pixel lanes per chunk
    const int q = tid % Q, r = tid / Q;
    const int per = (p.HW + kCaSplit - 1) / kCaSplit;
    const int px0 = sp * per, px1 = min(p.HW, px0 + per);
    const uint16_t* xb = p.x + (size_t)n * p.HW * p.xs + q * 8;
    if (r < rows) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int px = px0 + r; px < px1; px += rows) {
            float v[8];
            unpack8(*reinterpret_cast<const uint4*>(xb + (size_t)px * p.xs), v);
#pragma unroll
            for (int c = 0; c < 8; c++) acc[c] += v[c];
        }
#pragma unroll
        for (int c = 0; c < 8; c++) red[r * p.C + q * 8 + c] = acc[c];
    }
    __syncthreads();
    for (int c = tid; c < p.C; c += 256) {
        float sum = 0.f;
        for (int i = 0; i < rows; i++) sum += red[i * p.C + c];
        p.part[((size_t)n * kCaSplit + sp) * p.C + c] = sum;
    }
}

// One 64-lane workgroup per (image, 64 output channels): the C-long dot products keep their
// k order (one fmaf chain per output), with the weights loaded kCaBatch rows at a time ahead
// of the chain; one workgroup per image with one load per fmaf ran ~95 us per call at 128
// images (a load latency per k, half the CUs idle).
constexpr int kCaBatch = 8;

__global__ __launch_bounds__(64) void ca_fc_kernel(CaParams p) {
    extern __shared__ float mean[];  // [C]
    const int n = blockIdx.y, tid = threadIdx.x;
    for (int c = tid; c < p.C; c += 64) {
        float sum = 0.f;
        for (int i = 0; i < kCaSplit; i++) sum += p.part[((size_t)n * kCaSplit + i) * p.C + c];
        mean[c] = sum / (float)p.HW;
    }
    __syncthreads();
    const int c = blockIdx.x * 64 + tid;
    if (c >= p.C) return;
    float a = p.b[c];
    const float* wc = p.wt + c;
    int k = 0;
    for (; k + kCaBatch <= p.C; k += kCaBatch) {
        float w[kCaBatch];
#pragma unroll
        for (int j = 0; j < kCaBatch; j++) w[j] = wc[(size_t)(k + j) * p.C];
#pragma unroll
        for (int j = 0; j < kCaBatch; j++) a = fmaf(w[j], mean[k + j], a);
    }
    for (; k < p.C; k++) a = fmaf(wc[(size_t)k * p.C], mean[k], a);
    p.s[(size_t)n * p.C + c] = fminf(fmaxf(a + 3.f, 0.f), 6.f) / 6.f;
}

__global__ __launch_bounds__(256) void ca_scale_kernel(uint16_t* x, const float* s, int HW, int C, int xs) {
    const int n = blockIdx.y;
    const int Q = C / 8;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)HW * Q) return;
    const int px = (int)(i / Q), q = (int)(i - (long)px * Q);
    uint4* ptr = reinterpret_cast<uint4*>(x + ((size_t)n * HW + px) * xs + q * 8);
    float v[8];
    unpack8(*ptr, v);
    const float* sc = s + (size_t)n * C + q * 8;
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] *= sc[c];
    *ptr = pack8(v);
}

// ------------------------------------------------------------------ SPP max pools
// maxpool 9 = maxpool 5 twice, 13 = three times (stride 1, -inf padding: exact), so one
// workgroup per (image, G 8-channel groups) keeps the plane in LDS and applies the 5x5 max three
// times, writing each result into its slice.  The 5x5 max is a 5-wide row max, then a 5-tall
// column max of those (max is exact and order-free; every value is bf16, so the packed row
// maxima are exact too); the column max overwrites the plane it started from (the row maxima
// are a plane of their own).  G = 4 (round 6): a thread item is one 16-B chunk of a pixel, so a
// pixel's 64 B load and store coalesce and each phase has 6 items per thread instead of 1.6
// (one 8-channel group per workgroup ran 515 us for the 20x20 x 384 SPP of 512 frames).
template <int G>
__global__ __launch_bounds__(256) void spp_kernel(uint16_t* buf, int H, int W, int C, int xs) {
    extern __shared__ uint4 pl[];  // two planes [H*W][G]: the pooled input, its row maxima
    const int cg = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, HW = H * W, NI = HW * G;
    uint16_t* base = buf + (size_t)n * HW * xs + cg * 8 * G;
    uint4* a = pl;
    uint4* r = pl + NI;
    for (int i = tid; i < NI; i += 256) {
        const int px = i / G, g = i - px * G;
        a[i] = *reinterpret_cast<const uint4*>(base + (size_t)px * xs + g * 8);
    }
    for (int k = 1; k <= 3; k++) {
        __syncthreads();
        for (int i = tid; i < NI; i += 256) {
            const int px = i / G, g = i - px * G, y = px / W, x = px - y * W;
            float m[8];
            for (int c = 0; c < 8; c++) m[c] = -__builtin_inff();
            for (int xx = max(x - 2, 0); xx <= min(x + 2, W - 1); xx++) {
                float v[8];
                unpack8(a[(y * W + xx) * G + g], v);
#pragma unroll
                for (int c = 0; c < 8; c++) m[c] = fmaxf(m[c], v[c]);
            }
            r[i] = pack8(m);
        }
        __syncthreads();
        for (int i = tid; i < NI; i += 256) {
            const int px = i / G, g = i - px * G, y = px / W, x = px - y * W;
            float m[8];
            for (int c = 0; c < 8; c++) m[c] = -__builtin_inff();
            for (int yy = max(y - 2, 0); yy <= min(y + 2, H - 1); yy++) {
                float v[8];
                unpack8(r[(yy * W + x) * G + g], v);
#pragma unroll
                for (int c = 0; c < 8; c++) m[c] = fmaxf(m[c], v[c]);
            }
            const uint4 o = pack8(m);
            a[i] = o;
            *reinterpret_cast<uint4*>(base + (size_t)px * xs + k * C + g * 8) = o;
        }
    }
}

// ------------------------------------------------------------------ nearest 2x
__global__ __launch_bounds__(256) void up2_kernel(const uint16_t* x, int xs, uint16_t* y, int ys, int H, int W, int C) {
    const int n = blockIdx.y, Q = C / 8;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;  // output (pixel, chunk)
    if (i >= (long)4 * H * W * Q) return;
    const int px = (int)(i / Q), q = (int)(i - (long)px * Q);
    const int yo = px / (2 * W), xo = px - yo * (2 * W);
    const uint4 v = *reinterpret_cast<const uint4*>(x + ((size_t)n * H * W + (size_t)(yo >> 1) * W + (xo >> 1)) * xs + q * 8);
    *reinterpret_cast<uint4*>(y + ((size_t)n * 4 * H * W + px) * ys + q * 8) = v;
}

// ------------------------------------------------------------------ head predictions
// One thread per pixel of a level: rtm_cls (1) and rtm_reg (4) 1x1 convs on the [cls |
// reg] features (f32 dot products, weights in LDS), sigmoid score, exp(reg) * stride,
// prior (x, y) * stride, distance2bbox clipped to [0, size].
struct HeadParams {
    const uint16_t* x;  // [n][H][W] pixels of xs elements: cls feat at 0, reg feat at F
    const float* w;     // [5][F]
    const float* b;     // [5]
    float* cand;        // [n][n_priors][6]
    int H, W, F, xs, stride, size, n_priors, prior0;
};

__global__ __launch_bounds__(256) void det_head_kernel(HeadParams p) {
#pragma clang fp contract(off)  // box arithmetic rounded op by op, as mmdet's torch ops
    extern __shared__ float swh[];  // [5][F]
    const int n = blockIdx.y, tid = threadIdx.x;
    for (int i = tid; i < 5 * p.F; i += 256) swh[i] = p.w[i];
    __syncthreads();
    const int px = blockIdx.x * 256 + tid;
    if (px >= p.H * p.W) return;
    const uint16_t* xc = p.x + ((size_t)n * p.H * p.W + px) * p.xs;
    const uint16_t* xr = xc + p.F;
    float a[5] = {p.b[0], p.b[1], p.b[2], p.b[3], p.b[4]};
    for (int k = 0; k < p.F; k += 8) {
        float c[8], r[8];
        unpack8(*reinterpret_cast<const uint4*>(xc + k), c);
        unpack8(*reinterpret_cast<const uint4*>(xr + k), r);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a[0] = fmaf(swh[k + j], c[j], a[0]);
#pragma unroll
            for (int o = 1; o < 5; o++) a[o] = fmaf(swh[o * p.F + k + j], r[j], a[o]);
        }
    }
    const int yy = px / p.W, xx = px - yy * p.W;
    const float s = (float)p.stride;
    const float pxf = (float)xx * s, pyf = (float)yy * s;
    const float d0 = expf(a[1]) * s, d1 = expf(a[2]) * s, d2 = expf(a[3]) * s, d3 = expf(a[4]) * s;
    const float lim = (float)p.size;
    float* out = p.cand + ((size_t)n * p.n_priors + p.prior0 + px) * 6;
    out[0] = 1.f / (1.f + expf(-a[0]));
    out[1] = fminf(fmaxf(pxf - d0, 0.f), lim);
    out[2] = fminf(fmaxf(pyf - d1, 0.f), lim);
    out[3] = fminf(fmaxf(pxf + d2, 0.f), lim);
    out[4] = fminf(fmaxf(pyf + d3, 0.f), lim);
    out[5] = a[0];
}

// The same head with the features staged through LDS: a pixel's [cls | reg] channels sit
// xs elements apart, so one lane per pixel made every 16-B load instruction touch 64 rows
// (2.3 TB/s).  Here the workgroup's 256 pixels x 32 + 32 channels arrive as 64-B runs per
// pixel (coalesced), then each lane runs the same fmaf chains in the same k order.
constexpr int kHeadKC = 32;  // channels of cls and of reg per staging step

__global__ __launch_bounds__(256) void det_head_staged_kernel(HeadParams p) {
#pragma clang fp contract(off)  // box arithmetic rounded op by op, as mmdet's torch ops
    extern __shared__ float swh[];  // [5][F], then the pixel block [256][9] uint4
    uint4* sx = reinterpret_cast<uint4*>(swh + ((5 * p.F + 3) & ~3));
    const int n = blockIdx.y, tid = threadIdx.x;
    for (int i = tid; i < 5 * p.F; i += 256) swh[i] = p.w[i];
    const int HW = p.H * p.W, px0 = blockIdx.x * 256;
    const uint16_t* xb = p.x + (size_t)n * HW * p.xs;
    float a[5] = {p.b[0], p.b[1], p.b[2], p.b[3], p.b[4]};
    for (int kc = 0; kc < p.F; kc += kHeadKC) {
        __syncthreads();  // the previous step's block is consumed (and the weights are in)
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int i = tid + 256 * j, pl = i >> 3, q = i & 7;
            const int pg = min(px0 + pl, HW - 1);
            const int ch = q < 4 ? kc + 8 * q : p.F + kc + 8 * (q - 4);
            sx[pl * 9 + q] = *reinterpret_cast<const uint4*>(xb + (size_t)pg * p.xs + ch);
        }
        __syncthreads();
#pragma unroll
        for (int sq = 0; sq < kHeadKC / 8; sq++) {
            const int k = kc + 8 * sq;
            float c[8], r[8];
            unpack8(sx[tid * 9 + sq], c);
            unpack8(sx[tid * 9 + 4 + sq], r);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a[0] = fmaf(swh[k + j], c[j], a[0]);
#pragma unroll
                for (int o = 1; o < 5; o++) a[o] = fmaf(swh[o * p.F + k + j], r[j], a[o]);
            }
        }
    }
    const int px = px0 + tid;
    if (px >= HW) return;
    const int yy = px / p.W, xx = px - yy * p.W;
    const float s = (float)p.stride;
    const float pxf = (float)xx * s, pyf = (float)yy * s;
    const float d0 = expf(a[1]) * s, d1 = expf(a[2]) * s, d2 = expf(a[3]) * s, d3 = expf(a[4]) * s;
    const float lim = (float)p.size;
    float* out = p.cand + ((size_t)n * p.n_priors + p.prior0 + px) * 6;
    out[0] = 1.f / (1.f + expf(-a[0]));
    out[1] = fminf(fmaxf(pxf - d0, 0.f), lim);
    out[2] = fminf(fmaxf(pyf - d1, 0.f), lim);
    out[3] = fminf(fmaxf(pxf + d2, 0.f), lim);
    out[4] = fminf(fmaxf(pyf + d3, 0.f), lim);
    out[5] = a[0];
}

// ------------------------------------------------------------------ per-frame argmax
// The reference keeps the first detection after mmdet's NMS = the highest-scoring prior
// that passed score_thr and the min-size filter (NMS never removes the top box).  Ties go
// to the lowest prior index (level-major, row-major: the order of a stable sort).
__global__ __launch_bounds__(256) void det_select_kernel(const float* cand, int n_priors, float score_thr, float fx,
                                                         float fy, float* best) {
#pragma clang fp contract(off)
    __shared__ float ss[256];
    __shared__ int si[256];
    const int n = blockIdx.x, tid = threadIdx.x;
    float bs = -1.f;
    int bi = 0x7fffffff;
    for (int i = tid; i < n_priors; i += 256) {
        const float* c = cand + ((size_t)n * n_priors + i) * 6;
        const float s = c[0];
        const float x1 = c[1] * fx, y1 = c[2] * fy, x2 = c[3] * fx, y2 = c[4] * fy;
        if (s > score_thr && x2 - x1 > 0.f && y2 - y1 > 0.f && s > bs) bs = s, bi = i;  // i increases: first max kept
    }
    ss[tid] = bs;
    si[tid] = bi;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            const float s2 = ss[tid + w];
            const int i2 = si[tid + w];
            if (s2 > ss[tid] || (s2 == ss[tid] && i2 < si[tid])) ss[tid] = s2, si[tid] = i2;
        }
        __syncthreads();
    }
    if (tid == 0) {
        float* o = best + (size_t)n * 6;
        if (si[0] == 0x7fffffff) {
            o[0] = o[1] = o[2] = o[3] = 0.f;
            o[4] = -1.f;
            o[5] = -1.f;
        } else {
            const float* c = cand + ((size_t)n * n_priors + si[0]) * 6;
            o[0] = c[1] * fx, o[1] = c[2] * fy, o[2] = c[3] * fx, o[3] = c[4] * fy;
            o[4] = ss[0];
            o[5] = (float)si[0];
        }
    }
}

// ------------------------------------------------------------------ NMS (full list)
// One workgroup per frame.  Per level: the priors above score_thr are ranked by
// (score desc, index asc) with a bitonic sort of (score, index) keys in LDS and the best
// nms_pre kept; the survivors of all levels are rescaled, min-size filtered, sorted again
// and suppressed greedily (IoU > iou_thr, mmcv nms with offset 0).
constexpr int kNmsCap = 8192;  // keys per sort (a level's priors; <= 6400 at size 640)

__device__ void bitonic_desc(unsigned long long* k, int n_pow2) {
    for (int size = 2; size <= n_pow2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n_pow2; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;  // descending in "up" runs
                    const unsigned long long a = k[i], b = k[j];
                    if (up ? a < b : a > b) k[i] = b, k[j] = a;
                }
            }
        }
    __syncthreads();
}

// key: score bits (positive floats order as unsigned) high, inverted index low, so a
// descending sort puts higher score first and, for equal scores, the lower index first
__device__ __forceinline__ unsigned long long nms_key(float s, int i) {
    return ((unsigned long long)__float_as_uint(s) << 32) | (unsigned)(0x7fffffff - i);
}

__global__ __launch_bounds__(1024) void det_nms_kernel(const float* cand, int n_priors, const int* level_off, int n_levels,
                                                       int nms_pre, float score_thr, float iou_thr, int max_det, float fx,
                                                       float fy, float* dets, int* counts) {
#pragma clang fp contract(off)  // rescale / IoU rounded op by op (mmcv nms, offset 0)
    extern __shared__ unsigned long long keys[];  // [kNmsCap]
    __shared__ int n_sel;
    __shared__ int sel[3072];  // kept prior ids over the levels (nms_pre <= 1024 each, <= 3 levels)
    __shared__ float4 bx[3072];
    __shared__ float sc[3072];
    __shared__ unsigned char dead[3072];
    const int n = blockIdx.x, tid = threadIdx.x;
    const float* cn = cand + (size_t)n * n_priors * 6;
    if (tid == 0) n_sel = 0;
    for (int l = 0; l < n_levels; l++) {
        const int lo = level_off[l], cnt = level_off[l + 1] - lo;
        int np2 = 1;
        while (np2 < cnt) np2 <<= 1;
        for (int i = tid; i < np2; i += blockDim.x) {
            const float s = i < cnt ? cn[(size_t)(lo + i) * 6] : 0.f;
            keys[i] = (i < cnt && s > score_thr) ? nms_key(s, lo + i) : 0ull;
        }
        bitonic_desc(keys, np2);
        const int base = n_sel;
        for (int i = tid; i < nms_pre && i < np2; i += blockDim.x)
            if (keys[i] != 0ull) {
                const int idx = 0x7fffffff - (int)(keys[i] & 0xffffffffu);
                sel[base + i] = idx;
            } else {
                sel[base + i] = -1;
            }
        __syncthreads();
        if (tid == 0) {
            int k = base;
            for (int i = 0; i < nms_pre && i < np2; i++)
                if (sel[base + i] >= 0) sel[k++] = sel[base + i];
            n_sel = k;
        }
        __syncthreads();
    }
    const int m = n_sel;
    // rescale + min-size filter, then one global ranking of the survivors
    int np2 = 1;
    while (np2 < m) np2 <<= 1;
    for (int i = tid; i < np2; i += blockDim.x) {
        unsigned long long key = 0ull;
        if (i < m) {
            const float* c = cn + (size_t)sel[i] * 6;
            const float x1 = c[1] * fx, y1 = c[2] * fy, x2 = c[3] * fx, y2 = c[4] * fy;
            bx[i] = float4{x1, y1, x2, y2};
            sc[i] = c[0];
            if (x2 - x1 > 0.f && y2 - y1 > 0.f) key = nms_key(c[0], i);
        }
        keys[i] = key;
    }
    bitonic_desc(keys, np2);
    for (int i = tid; i < m; i += blockDim.x) dead[i] = 0;
    __syncthreads();
    int kept = 0;
    float* out = dets + (size_t)n * max_det * 5;
    for (int a = 0; a < m && kept < max_det; a++) {
        const unsigned long long ka = keys[a];
        if (ka == 0ull) break;
        const int ia = 0x7fffffff - (int)(ka & 0xffffffffu);
        if (dead[a]) continue;  // uniform: every thread reads the same flag after the barrier
        const float4 A = bx[ia];
        if (tid == 0) {
            float* o = out + (size_t)kept * 5;
            o[0] = A.x, o[1] = A.y, o[2] = A.z, o[3] = A.w, o[4] = sc[ia];
        }
        kept++;
        const float area_a = (A.z - A.x) * (A.w - A.y);
        for (int b = a + 1 + tid; b < m; b += blockDim.x) {
            const unsigned long long kb = keys[b];
            if (kb == 0ull || dead[b]) continue;
            const float4 B = bx[0x7fffffff - (int)(kb & 0xffffffffu)];
            const float w = fmaxf(fminf(A.z, B.z) - fmaxf(A.x, B.x), 0.f);
            const float h = fmaxf(fminf(A.w, B.w) - fmaxf(A.y, B.y), 0.f);
            const float inter = w * h;
            const float iou = inter / (area_a + (B.z - B.x) * (B.w - B.y) - inter);
            if (iou > iou_thr) dead[b] = 1;
        }
        __syncthreads();
    }
    if (tid == 0) counts[n] = kept;
}

// ------------------------------------------------------------------ depthwise 5x5 + pointwise 1x1
// One CSPNeXtBlock's conv2 (DepthwiseSeparableConvModule: 5x5 depthwise + BN + SiLU, then 1x1
// pointwise + BN + SiLU, + the block's identity) in one launch: the depthwise output never leaves
// LDS.  Unfused, dw5_kernel wrote it (C channels per pixel) and the 1x1 GEMM read it back: 2 x C x
// 2 B per pixel of HBM traffic and a launch per block, ~37 % of the pair's bytes.
// A workgroup owns a TH x TW pixel tile of one frame and all C channels:
//   dw phase   8-channel chunks, 8 per round (one per wave): the round's (TH+4) x (TW+4) halo
//              is loaded coalesced into LDS (8 consecutive 16-B chunks of a pixel per lane
//              group, dw5_kernel's layout), each wave computes its chunk for the tile (1 or 2
//              outputs per lane: dw5_kernel's fma chains, taps in (kh, kw) order, packed
//              channel pairs) and writes the bf16 result straight into the GEMM's B operand;
//   pw phase   the tile x C couts GEMM on v_mfma_f32_16x16x32_bf16 with the B operand resident
//              for all C/32 K steps and the weight image (det_pack_gemm_weights) streamed per K
//              step through a 2-slot LDS ring (register-staged: step q+2 loads under step q);
//              waves split pixel fragments x cout tiles;
//   epilogue   det_conv_gemm_kernel's: bias, SiLU, + residual, bf16.
// Bit-identical to dw5_kernel + det_conv_gemm_kernel<*, 1, 1>: the same per-output fma chains,
// bf16 rounding of the intermediate, LDS operand layouts (row-major 16-B slots with chunk
// kg at kg ^ swz(row)), MFMA operand roles and K order (tests/test_rtmdet_gpu.py).
struct DwPwParams {
    const uint16_t* x;      // depthwise input view (pixel stride xs)
    const float* dw_w;      // [C/8][25][8]
    const float* dw_b;      // [C]
    const uint16_t* wimg;   // pointwise weight image: [C/32 K steps][C couts][4 swizzled 16-B chunks]
    const float* pw_b;      // [C]
    const uint16_t* res;    // residual view (stride rs) or nullptr
    uint16_t* y;            // output view (stride ys)
    int H, W, N, xs, ys, rs, act_dw, act_pw, tiles_w;
};

template <int C, int TH_, int TW>
struct DwPwCfg {
    static constexpr int TH = TH_, P = TH * TW, OUTS = P / 64;  // dw outputs per lane
    static constexpr int HH = TH + 4, HWD = TW + 4;           // halo rows / columns
    static constexpr int Q = C / 32, NCH = C / 8;             // K steps, 8-channel chunks
    static constexpr int FP = P / 16, NT = C / 16;            // pixel fragments, cout tiles
    static constexpr int PWV = FP < 8 ? FP : 8, CWV = 8 / PWV;
    static constexpr int FPW = FP / PWV, TPW = NT / CWV;      // per wave
    static constexpr int B_BYTES = Q * P * 64, A_BYTES = C * 64, H_BYTES = HH * HWD * 8 * 16;
    static constexpr int LDS = B_BYTES + 2 * A_BYTES + H_BYTES;
    static constexpr int AR = (C * 4 + 511) / 512;            // weight chunks per thread and K step
    static_assert(FP % PWV == 0 && NT % CWV == 0 && (OUTS == 1 || OUTS == 2), "dwpw tiling");
};

template <int C, int TH, int TW>
__global__ __launch_bounds__(512, TH == 4 ? 3 : 2) void dwpw_kernel(DwPwParams p) {
    using G = DwPwCfg<C, TH, TW>;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* Bt = lds;                        // [Q][P rows][4 slots]
    uint8_t* At = lds + G::B_BYTES;           // 2 x [C rows][4 slots]
    uint4* halo = reinterpret_cast<uint4*>(lds + G::B_BYTES + 2 * G::A_BYTES);  // [8 chunks][HH * HWD]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int th = blockIdx.x / p.tiles_w, tw = blockIdx.x - th * p.tiles_w;
    const int n = blockIdx.y;
    const int h0 = th * G::TH, w0 = tw * TW;
    auto swz = [](int r) { return (-(r >> 2)) & 3; };
    // weight ring: step q's C x 64 B slab is contiguous in the image
    uint4 wr[G::AR];
    auto load_w = [&](int q) {
#pragma unroll
        for (int j = 0; j < G::AR; j++) {
            const int i = tid + j * 512;
            if (i < C * 4) wr[j] = *reinterpret_cast<const uint4*>(p.wimg + ((size_t)q * C * 4 + i) * 8);
        }
    };
    auto store_w = [&](int slot) {
#pragma unroll
        for (int j = 0; j < G::AR; j++) {
            const int i = tid + j * 512;
            if (i < C * 4) *reinterpret_cast<uint4*>(At + slot * G::A_BYTES + i * 16) = wr[j];
        }
    };
    load_w(0);
    // the epilogue's residual, loaded now so that it lands under the depthwise phase
    const int wp = wave % G::PWV, wc = wave / G::PWV;
    const int kg = lane >> 4, r16 = lane & 15;
    uint2 rsd[G::FPW][G::TPW];
    if (p.res) {
#pragma unroll
        for (int i = 0; i < G::FPW; i++) {
            const int px = (wp * G::FPW + i) * 16 + r16;
            const int h = h0 + px / TW, w = w0 + px % TW;
#pragma unroll
            for (int j = 0; j < G::TPW; j++) {
                const int co = (wc * G::TPW + j) * 16 + kg * 4;
                rsd[i][j] = (h < p.H && w < p.W && co < p.N)
                                ? *reinterpret_cast<const uint2*>(p.res + (((size_t)n * p.H + h) * p.W + w) * p.rs + co)
                                : uint2{0u, 0u};
            }
        }
    }
    // ---- depthwise phase
    const uint16_t* xb = p.x + (size_t)n * p.H * p.W * p.xs;
    typedef float f32x2v __attribute__((ext_vector_type(2)));
#pragma unroll 1
    for (int c0 = 0; c0 < G::NCH; c0 += 8) {
        const int g = min(8, G::NCH - c0);   // chunks this round
        {   // every load of the round in flight before the first LDS write
            constexpr int HR = (G::HH * G::HWD * 8 + 511) / 512;
            uint4 hv[HR];
#pragma unroll
            for (int j = 0; j < HR; j++) {
                const int i = tid + j * 512;
                hv[j] = uint4{0u, 0u, 0u, 0u};
                if (i < G::HH * G::HWD * g) {
                    const int pix = i / g, q = i - pix * g;
                    const int r = pix / G::HWD, c = pix - r * G::HWD;
                    const int hi = h0 - 2 + r, wi = w0 - 2 + c;
                    if (hi >= 0 && hi < p.H && wi >= 0 && wi < p.W)
                        hv[j] = *reinterpret_cast<const uint4*>(xb + ((size_t)hi * p.W + wi) * p.xs + (c0 + q) * 8);
                }
            }
#pragma unroll
            for (int j = 0; j < HR; j++) {
                const int i = tid + j * 512;
                if (i < G::HH * G::HWD * g) {
                    const int pix = i / g, q = i - pix * g;
                    halo[q * G::HH * G::HWD + pix] = hv[j];
                }
            }
        }
        __syncthreads();
        if (wave < g) {
            const int chunk = c0 + wave;
            const float* wc = p.dw_w + (size_t)chunk * 200;
            const float* bc = p.dw_b + chunk * 8;
            const uint4* hq = halo + wave * G::HH * G::HWD;
            const int q = chunk >> 2, kg = chunk & 3;
            if constexpr (G::OUTS == 2) {   // dw5_kernel's lane layout: 2 vertical outputs per lane
                const int col = lane & 15, rp = lane >> 4;
                f32x2v a0[4], a1[4];
#pragma unroll
                for (int c = 0; c < 4; c++) a0[c] = a1[c] = f32x2v{0.f, 0.f};
#pragma unroll 1
                for (int ir = 0; ir < 6; ir++) {
#pragma unroll
                    for (int kw = 0; kw < 5; kw++) {
                        float v[8];
                        unpack8(hq[(2 * rp + ir) * G::HWD + col + kw], v);
                        if (ir < 5) {
                            const float* wk = wc + (ir * 5 + kw) * 8;
#pragma unroll
                            for (int c = 0; c < 4; c++)
                                a0[c] = __builtin_elementwise_fma(f32x2v{v[2 * c], v[2 * c + 1]},
                                                                  f32x2v{wk[2 * c], wk[2 * c + 1]}, a0[c]);
                        }
                        if (ir >= 1) {
                            const float* wk = wc + ((ir - 1) * 5 + kw) * 8;
#pragma unroll
                            for (int c = 0; c < 4; c++)
                                a1[c] = __builtin_elementwise_fma(f32x2v{v[2 * c], v[2 * c + 1]},
                                                                  f32x2v{wk[2 * c], wk[2 * c + 1]}, a1[c]);
                        }
                    }
                }
                float o0[8], o1[8];
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    o0[c] = act_f(a0[c >> 1][c & 1] + bc[c], p.act_dw);
                    o1[c] = act_f(a1[c >> 1][c & 1] + bc[c], p.act_dw);
                }
                const int pa = (2 * rp) * TW + col, pb = pa + TW;
                *reinterpret_cast<uint4*>(Bt + q * G::P * 64 + pa * 64 + ((kg ^ swz(pa)) * 16)) = pack8(o0);
                *reinterpret_cast<uint4*>(Bt + q * G::P * 64 + pb * 64 + ((kg ^ swz(pb)) * 16)) = pack8(o1);
            } else {                          // one output per lane, the same chain (taps in (kh, kw) order)
                const int col = lane % TW, row = lane / TW;
                f32x2v a0[4];
#pragma unroll
                for (int c = 0; c < 4; c++) a0[c] = f32x2v{0.f, 0.f};
#pragma unroll 1
                for (int kh = 0; kh < 5; kh++) {
#pragma unroll
                    for (int kw = 0; kw < 5; kw++) {
                        float v[8];
                        unpack8(hq[(row + kh) * G::HWD + col + kw], v);
                        const float* wk = wc + (kh * 5 + kw) * 8;
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            a0[c] = __builtin_elementwise_fma(f32x2v{v[2 * c], v[2 * c + 1]},
                                                              f32x2v{wk[2 * c], wk[2 * c + 1]}, a0[c]);
                    }
                }
                float o0[8];
#pragma unroll
                for (int c = 0; c < 8; c++) o0[c] = act_f(a0[c >> 1][c & 1] + bc[c], p.act_dw);
                const int pa = row * TW + col;
                *reinterpret_cast<uint4*>(Bt + q * G::P * 64 + pa * 64 + ((kg ^ swz(pa)) * 16)) = pack8(o0);
            }
        }
        __syncthreads();   // the halo is reloaded by the next round
    }
    store_w(0);
    if (G::Q > 1) load_w(1);
    __syncthreads();
    // ---- pointwise phase
    const int soff = r16 * 64 + ((kg ^ swz(r16)) * 16);
    f32x4 acc[G::FPW][G::TPW];
#pragma unroll
    for (int i = 0; i < G::FPW; i++)
#pragma unroll
        for (int j = 0; j < G::TPW; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int q = 0; q < G::Q; q++) {
        const uint8_t* ab = At + (q & 1) * G::A_BYTES;
        const uint8_t* bb = Bt + q * G::P * 64;
        bf16x8 a[G::TPW], b[G::FPW];
#pragma unroll
        for (int j = 0; j < G::TPW; j++)
            a[j] = *reinterpret_cast<const bf16x8*>(ab + ((wc * G::TPW + j) * 16) * 64 + soff);
#pragma unroll
        for (int i = 0; i < G::FPW; i++)
            b[i] = *reinterpret_cast<const bf16x8*>(bb + ((wp * G::FPW + i) * 16) * 64 + soff);
#pragma unroll
        for (int i = 0; i < G::FPW; i++)
#pragma unroll
            for (int j = 0; j < G::TPW; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[i], acc[i][j], 0, 0, 0);
        if (q + 1 < G::Q) {
            store_w((q + 1) & 1);   // that slot was last read in step q - 1: every wave is past it
            if (q + 2 < G::Q) load_w(q + 2);
        }
        __syncthreads();
    }
    // ---- epilogue (det_conv_gemm_kernel's)
#pragma unroll
    for (int j = 0; j < G::TPW; j++) {
        const int co = (wc * G::TPW + j) * 16 + kg * 4;
        if (co >= p.N) continue;
        const float4 bb = *reinterpret_cast<const float4*>(p.pw_b + co);
#pragma unroll
        for (int i = 0; i < G::FPW; i++) {
            const int px = (wp * G::FPW + i) * 16 + r16;
            const int h = h0 + px / TW, w = w0 + px % TW;
            if (h >= p.H || w >= p.W) continue;
            const size_t m = ((size_t)n * p.H + h) * p.W + w;
            float v[4] = {acc[i][j][0] + bb.x, acc[i][j][1] + bb.y, acc[i][j][2] + bb.z, acc[i][j][3] + bb.w};
            if (p.act_pw == 2)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = act_f(v[e], 2);
            if (p.res) {
                const uint2 r = rsd[i][j];
                v[0] += bf(r.x & 0xffff), v[1] += bf(r.x >> 16), v[2] += bf(r.y & 0xffff), v[3] += bf(r.y >> 16);
            }
            if (p.act_pw == 1)
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] = fmaxf(v[e], 0.f);
            *reinterpret_cast<uint2*>(p.y + m * p.ys + co) =
                uint2{tobf(v[0]) | (tobf(v[1]) << 16), tobf(v[2]) | (tobf(v[3]) << 16)};
        }
    }
}

}  // namespace

// ---------------------------------------------------------------------------- launchers
namespace {
LbParams lb_params(const uint8_t* frames, int H, int W, int S, const float* mean3, const float* std3, void* out) {
    int nh, nw;
    det_rescale_size(H, W, S, nh, nw);
    MVP_REQUIRE(nh >= 1 && nw >= 1 && nh <= S && nw <= S, "letterbox: bad size");
    LbParams p{};
    p.f = frames;
    p.out = static_cast<uint32_t*>(out);
    p.H = H, p.W = W, p.S = S, p.nh = nh, p.nw = nw;
    p.scale_x = 1.0 / ((double)nw / W);
    p.scale_y = 1.0 / ((double)nh / H);
    p.area2 = p.scale_x == 2.0 && p.scale_y == 2.0 && W == 2 * nw && H == 2 * nh;
    for (int c = 0; c < 3; c++) p.mean[c] = mean3[c], p.stdv[c] = std3[c];
    return p;
}
}  // namespace

void launch_det_letterbox(const uint8_t* frames, int n, int H, int W, int S, const float* mean3, const float* std3,
                          void* out, hipStream_t s) {
    const LbParams p = lb_params(frames, H, W, S, mean3, std3, out);
    if (n == 0) return;
    hipLaunchKernelGGL(letterbox_kernel, dim3((unsigned)((S * S + 255) / 256), (unsigned)n), dim3(256), 0, s, p);
    MVP_HIP(hipGetLastError());
}

void det_rescale_size(int H, int W, int S, int& nh, int& nw) {
    const double sc = std::min((double)S / std::max(H, W), (double)S / std::min(H, W));
    nh = (int)(H * sc + 0.5);
    nw = (int)(W * sc + 0.5);
}

namespace {
void stem_launch(const uint16_t* x, const float* w, const float* b, uint16_t* y, int n, int S, int act, hipStream_t s,
                 const LbParams* lb) {
    MVP_REQUIRE(S % 16 == 0, "det stem: size %d must be a multiple of 16", S);
    const long n_tiles = (long)n * (S / 4);
    if (n_tiles == 0) return;
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const size_t lds = (size_t)5 * (S + 2) * sizeof(uint2);
    const long grid = std::min<long>(n_tiles, (long)cus * 8);
    if (lb)
        hipLaunchKernelGGL(det_stem_kernel<true>, dim3((unsigned)grid), dim3(256), lds, s, x, w, b, y, S, act, n_tiles, *lb);
    else
        hipLaunchKernelGGL(det_stem_kernel<false>, dim3((unsigned)grid), dim3(256), lds, s, x, w, b, y, S, act, n_tiles,
                           LbParams{});
    MVP_HIP(hipGetLastError());
}
}  // namespace

void launch_det_stem(const uint16_t* x, const float* w, const float* b, uint16_t* y, int n, int S, int act,
                     hipStream_t s) {
    stem_launch(x, w, b, y, n, S, act, s, nullptr);
}

void launch_det_letterbox_stem(const uint8_t* frames, int H, int W, const float* mean3, const float* std3,
                               const float* w, const float* b, uint16_t* y, int n, int S, int act, hipStream_t s) {
    const LbParams lb = lb_params(frames, H, W, S, mean3, std3, nullptr);
    stem_launch(nullptr, w, b, y, n, S, act, s, &lb);
}

void launch_det_dw5(const uint16_t* x, int xs, uint16_t* y, int ys, const float* w, const float* b, int n, int H, int W,
                    int C, int act, hipStream_t s) {
    MVP_REQUIRE(C % 32 == 0 && xs % 8 == 0 && ys % 8 == 0, "dw5: channels must be a multiple of 32");
    DwParams p{x, y, w, b, H, W, C, xs, ys, act, (W + kDwTW - 1) / kDwTW};
    // G chunks of 8 channels per workgroup: 8 (128 B of every pixel, one cache line), else 4.
    // (Measured: the 96-channel planes with all 12 chunks per workgroup read 1.37x the
    // algorithmic bytes instead of 2.07x but ran 555 vs 509 us per 80x80 layer of 512 frames,
    // gpurun_out/detbd3: 768-thread workgroups halve the occupancy.  Those planes now run fused,
    // dwpw_kernel.)
    const int G = C % 64 == 0 ? 8 : 4;
    const long blocks = (long)p.tiles_w * ((H + kDwTH - 1) / kDwTH) * (C / (8 * G));
    if (n == 0 || blocks == 0) return;
    MVP_REQUIRE(blocks < (1L << 31) && n < 65536, "dw5: grid too large");
    if (G == 8)
        hipLaunchKernelGGL(dw5_kernel<8>, dim3((unsigned)blocks, (unsigned)n), dim3(512), 0, s, p);
    else
        hipLaunchKernelGGL(dw5_kernel<4>, dim3((unsigned)blocks, (unsigned)n), dim3(256), 0, s, p);
    MVP_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void det_pack_gemm_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ img,
                                                          int npad, int K) {
    const long n = (long)npad * K / 8;  // 16-B slots
    for (long d = blockIdx.x * 256L + threadIdx.x; d < n; d += (long)gridDim.x * 256) {
        const long qc = d >> 2;  // (K step, cout)
        const int c = (int)(d & 3), co = (int)(qc % npad), q = (int)(qc / npad);
        const int kg = c ^ ((-(co >> 2)) & 3);  // the GEMM kernel's swz(co): co0 is a multiple of 16
        *reinterpret_cast<uint4*>(img + d * 8) =
            *reinterpret_cast<const uint4*>(w + (size_t)co * K + (size_t)q * 32 + kg * 8);
    }
}

void det_pack_gemm_weights(const uint16_t* w, uint16_t* img, int npad, int K, hipStream_t s) {
    MVP_REQUIRE(npad % 32 == 0 && K % 32 == 0, "det_pack_gemm_weights: npad %d, K %d", npad, K);
    hipLaunchKernelGGL(det_pack_gemm_kernel, dim3(512), dim3(256), 0, s, w, img, npad, K);
    MVP_HIP(hipGetLastError());
}

bool det_band_eligible(int H, int W, int cin, int npad, int ks, int stride) {
    return ks == 3 && stride == 1 && H == W && (W == 80 || W == 40) && cin % 32 == 0 && cin / 32 >= 3 &&
           npad % 32 == 0 && npad <= 32 * kBandBN;
}

int det_band_rows(int npad) { return (npad + kBandBN - 1) / kBandBN * kBandBN; }

void det_pack_band_weights(const uint16_t* w, uint16_t* img, int npad, int cin, hipStream_t s) {
    MVP_REQUIRE(npad % 32 == 0 && cin % 32 == 0, "det_pack_band_weights: npad %d, cin %d", npad, cin);
    hipLaunchKernelGGL(det_pack_band_kernel, dim3(512), dim3(256), 0, s, w, img, npad, cin);
    MVP_HIP(hipGetLastError());
}

namespace {
int g_det_cus = 0;

// one workgroup per CU, a multiple of 8 (the XCD round robin of blockIdx)
int det_band_grid() {
    if (g_det_cus == 0) {
        int dev = 0;
        MVP_HIP(hipGetDevice(&dev));
        MVP_HIP(hipDeviceGetAttribute(&g_det_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    return std::max(8, g_det_cus / 8 * 8);
}

template <int W, int TR, int NWV>
void launch_band(const GParams& p, const uint16_t* wband, hipStream_t s) {
    using C = BandCfg<W, TR>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)det_conv_band_kernel<W, TR, NWV>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
        attr = true;
    }
    const int grid = det_band_grid();
    hipLaunchKernelGGL((det_conv_band_kernel<W, TR, NWV>), dim3(grid), dim3(64 * NWV), C::LDS, s, p, wband);
}
}  // namespace

// the persistent halo kernel (A/B and tests: MVPOSE_DET_HALO_PERS=0 = det_conv_halo_kernel)
bool halo_pers_on() {
    const char* e = getenv("MVPOSE_DET_HALO_PERS");
    return !(e && e[0] == '0');
}

namespace {
bool det_pers_1x1_on() {
    const char* e = getenv("MVPOSE_DET_PERS");
    return !(e && e[0] == '0');
}
int det_conv_bn(int npad) {
    return npad % 192 == 0 ? 192 : npad % 128 == 0 ? 128 : npad % 96 == 0 ? 96 : npad % 64 == 0 ? 64 : 32;
}
}  // namespace

namespace {
// the shapes the fold kernels take (no environment: the graph decided at create time)
bool fold_shape_ok(int H, int W, int cin, int N, int ks, bool ca) {
    if (ks != 1 || N > kPersMaxN || cin % 32 != 0) return false;
    const int bn = det_conv_bn(det_cout_pad(N));
    if (bn != 192 && bn != 96) return false;  // the instantiated fold kernels
    // a 128-pixel tile's rows span at most 8 frames (the scale table)
    const long hw = (long)H * W;
    return hw > 0 && (!ca || (127 + hw - 1) / hw + 1 <= 8);
}
}  // namespace

bool det_conv_fold_ok(int H, int W, int cin, int N, int ks, bool ca) {
    const char* e = getenv("MVPOSE_DET_FOLD");
    return !(e && e[0] == '0') && det_pers_1x1_on() && fold_shape_ok(H, W, cin, N, ks, ca);
}

void launch_det_conv_gemm(const uint16_t* x, int xs, const uint16_t* w, const float* bias, const uint16_t* res, int rs,
                          uint16_t* y, int ys, int n, int H, int W, int cin, int N, int ks, int stride, int act,
                          hipStream_t s, const uint16_t* wimg, const uint16_t* wband, int live, const DetConvFold* fold) {
    if (live <= 0 || live > N) live = N;
    const int fm = fold ? (fold->up ? 1 : 0) | (fold->ca ? 2 : 0) : 0;
    if (fm) {
        MVP_REQUIRE(wimg && fold_shape_ok(H, W, cin, N, ks, fm & 2), "det conv: fold on a conv the fold kernels do not take");
        MVP_REQUIRE(fm != 3, "det conv: one fold per conv");
        MVP_REQUIRE(!(fm & 1) || (H % 2 == 0 && W % 2 == 0 && fold->up_c % 32 == 0 && fold->up_c <= cin &&
                                  fold->up_s % 8 == 0),
                    "det conv: upsample fold shape");
    }
    MVP_REQUIRE(cin % 32 == 0 && N % 4 == 0 && xs % 8 == 0 && ys % 4 == 0 && (!res || rs % 4 == 0),
                "det conv: cin=%d cout=%d strides %d/%d", cin, N, xs, ys);
    MVP_REQUIRE((ks == 1 && stride == 1) || (ks == 3 && (stride == 1 || stride == 2)), "det conv: ks %d stride %d", ks,
                stride);
    const int pad = ks / 2;
    const int Ho = (H + 2 * pad - ks) / stride + 1, Wo = (W + 2 * pad - ks) / stride + 1;
    const int npad = det_cout_pad(N);
    // cout tile: the widest of 192 / 128 / 96 / 64 dividing the padded couts.  Measured
    // alternatives, all slower on RTMDet-m (profiles/r03detcfg.txt, 128 frames, same box):
    // 128-cout tiles 27.2-27.5 vs 25.9 ms, 256-pixel tiles of 8 waves 27.7, of 4 waves 32.6,
    // a 4-slot ring level; removed with their environment switches in round 3.  Round 6
    // re-measured 256-pixel tiles on the <= 40x40 planes' 192-cout convs only (their 128-pixel
    // tiles re-read each weight slice 1.7-6.6x): 84.5 vs 81.2 ms per 512 frames, removed again
    // (profiles/r06_det_wide_live_ab.txt).
    const int bn = det_conv_bn(npad);
    GParams p{x, w, bias, res, y, conv_zero_region(), (long)n * Ho * Wo, cin, N, npad, xs, ys, rs, act,
              (npad + bn - 1) / bn, 0, H, W, Ho, Wo, wimg};
    if (fm) p.up = fold->up, p.up_s = fold->up_s, p.up_c = fold->up_c, p.ca = fold->ca;
    {
        const char* e = getenv("MVPOSE_DET_XCD");  // A/B: 0 = blockIdx order
        p.xcd_order = !(e && e[0] == '0');
    }
    // band-halo kernel for the 3x3/s1 convs with >= 96 input channels on the 80x80 / 40x40
    // planes (det_conv_band_kernel)
    // The kernel splits each XCD's grid/8 workgroups into groups of n_nb (one per cout block):
    // a part with fewer than 8 * n_nb CUs would get no group at all, so it takes the GEMM path.
    if (wband && det_band_eligible(H, W, cin, npad, ks, stride) &&
        det_band_rows(npad) / kBandBN <= det_band_grid() / 8) {
        const char* e = getenv("MVPOSE_DET_BAND");  // tests: 0 = the im2col GEMM kernel
        if (!(e && e[0] == '0')) {
            if (n == 0) return;
            GParams pb = p;
            pb.n_nb = det_band_rows(npad) / kBandBN;
            MVP_REQUIRE((long)n * H / (W == 80 ? 4 : 8) < (1L << 24), "det band conv: too many bands");
            // 8 waves (two per SIMD) by default: 22.30 vs 23.33 ms per 128-frame forward with 4
            // (gpurun_out/detband5); MVPOSE_DET_BAND=4 keeps the 4-wave form (tests: bit-identical)
            const bool w4 = e && e[0] == '4';
            if (W == 80) w4 ? launch_band<80, 4, 4>(pb, wband, s) : launch_band<80, 4, 8>(pb, wband, s);
            else w4 ? launch_band<40, 8, 4>(pb, wband, s) : launch_band<40, 8, 8>(pb, wband, s);
            MVP_HIP(hipGetLastError());
            return;
        }
    }
    // halo-tile kernel for the 32- and 64-channel 3x3/s1 convs (<= 64 couts): 14.03 -> 13.77
    // and 13.90 -> 13.86 ms per 64 frames against the im2col GEMM (same-box tools/det_ab.sh)
    if (ks == 3 && stride == 1 && (cin == 32 || cin == 64) && npad <= 64) {
        const char* e = getenv("MVPOSE_DET_HALO_ROWS");  // tests: 2 = the 2-row tiles
        const int tr = (e && e[0] == '2') ? 2 : DET_HALO_TR;
        const long tiles = (long)n * ((H + tr - 1) / tr) * ((W + 63) / 64);
        MVP_REQUIRE(tiles < (1L << 31), "det conv: grid too large");
        if (tiles == 0) return;
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), 0, s, p); };
        if (tr == 2) {
            if (cin == 64 && npad == 64) go(det_conv_halo_kernel<64, 2, 2>);
            else if (cin == 64) go(det_conv_halo_kernel<32, 2, 2>);
            else if (npad == 64) go(det_conv_halo_kernel<64, 1, 2>);
            else go(det_conv_halo_kernel<32, 1, 2>);
        } else if (npad == 64 && (live == 48 || live == 64) && !res && halo_pers_on()) {
            // persistent, weights resident (det_conv_halo_pers_kernel)
            auto go_p = [&](auto kern, int lds_bytes) {
                static int attr_done[4] = {0, 0, 0, 0};
                const int slot = (cin == 64) * 2 + (live == 64);
                if (!attr_done[slot]) {
                    MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
                    attr_done[slot] = 1;
                }
                const long T = (long)n * ((H + 7) / 8) * ((W + 63) / 64), cap = det_band_grid();
                const long grid = T <= cap ? T : cap / 8 * 8;
                hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds_bytes, s, p);
            };
            if (cin == 64 && live == 48) go_p(det_conv_halo_pers_kernel<64, 2, 3>, HaloPersCfg<64, 2, 3>::LDS);
            else if (cin == 64) go_p(det_conv_halo_pers_kernel<64, 2, 4>, HaloPersCfg<64, 2, 4>::LDS);
            else if (live == 48) go_p(det_conv_halo_pers_kernel<64, 1, 3>, HaloPersCfg<64, 1, 3>::LDS);
            else go_p(det_conv_halo_pers_kernel<64, 1, 4>, HaloPersCfg<64, 1, 4>::LDS);
        } else if (npad == 32 && cin == 32 && live > 16 && !res && halo_pers_on()) {
            // RTMDet-m stem.1 (24 -> 24 couts stored as 32): both 16-cout tiles live
            static bool attr32 = false;
            using G32 = HaloPersCfg<32, 1, 2>;
            if (!attr32) {
                MVP_HIP(hipFuncSetAttribute((const void*)det_conv_halo_pers_kernel<32, 1, 2>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, G32::LDS));
                attr32 = true;
            }
            const long T = (long)n * ((H + 7) / 8) * ((W + 63) / 64), cap = det_band_grid();
            const long grid = T <= cap ? T : cap / 8 * 8;
            hipLaunchKernelGGL((det_conv_halo_pers_kernel<32, 1, 2>), dim3((unsigned)grid), dim3(512), G32::LDS, s, p);
        } else if (npad == 64 && live <= 48 && live > 32 && !res && DET_HALO_TR % 4 == 0 &&
                   !(getenv("MVPOSE_DET_LIVE") && getenv("MVPOSE_DET_LIVE")[0] == '0')) {
            // 48 real couts in 64 (RTMDet-m stem.2, stage-1 conv1): 3 live tiles
            if (cin == 64) go(det_conv_halo_kernel<64, 2, DET_HALO_TR, 3>);
            else go(det_conv_halo_kernel<64, 1, DET_HALO_TR, 3>);
        } else {
            if (cin == 64 && npad == 64) go(det_conv_halo_kernel<64, 2, DET_HALO_TR>);
            else if (cin == 64) go(det_conv_halo_kernel<32, 2, DET_HALO_TR>);
            else if (npad == 64) go(det_conv_halo_kernel<64, 1, DET_HALO_TR>);
            else go(det_conv_halo_kernel<32, 1, DET_HALO_TR>);
        }
        MVP_HIP(hipGetLastError());
        return;
    }
    constexpr int kPx = 128;  // pixels per tile: 2 pixel waves x 4 fragments of 16
    const long blocks = (p.M + kPx - 1) / kPx * p.n_nb;
    if (blocks == 0) return;
    MVP_REQUIRE(blocks < (1L << 31), "det conv: grid too large");
    if (fm) {  // folds: the persistent 1x1 GEMM, whatever MVPOSE_DET_PERS now says (decided at create)
        const char* eo = getenv("MVPOSE_DET_PERS_OCC");
        const long occ = eo ? std::max(1, atoi(eo)) : 2;
        const long grid = blocks <= occ * det_band_grid() ? blocks : occ * det_band_grid() / 8 * 8;
        const dim3 gp((unsigned)grid), tp(256);
        if (fm == 1 && bn == 192) hipLaunchKernelGGL((det_conv1x1_pers_kernel<192, 1, 3, 1, 1, 1>), gp, tp, 0, s, p);
        else if (fm == 1) hipLaunchKernelGGL((det_conv1x1_pers_kernel<96, 2, 3, 1, 1, 1>), gp, tp, 0, s, p);
        else if (bn == 192) hipLaunchKernelGGL((det_conv1x1_pers_kernel<192, 1, 3, 1, 1, 2>), gp, tp, 0, s, p);
        else hipLaunchKernelGGL((det_conv1x1_pers_kernel<96, 2, 3, 1, 1, 2>), gp, tp, 0, s, p);
        MVP_HIP(hipGetLastError());
        return;
    }
    if (wimg && N <= kPersMaxN) {  // persistent GEMM: 2 workgroups per CU
        // A/B and tests: 0 = one tile per workgroup everywhere; 3 = the 3x3 GEMM convs too
        const char* e = getenv("MVPOSE_DET_PERS");
        if (det_pers_1x1_on() && (ks == 1 || (e && e[0] == '3'))) {
            // all blocks, or a multiple of 8 (the kernel's per-XCD split needs one of the two)
            const char* eo = getenv("MVPOSE_DET_PERS_OCC");  // A/B: workgroups per CU (default 2)
            const long occ = eo ? std::max(1, atoi(eo)) : 2;
            const long grid = blocks <= occ * det_band_grid() ? blocks : occ * det_band_grid() / 8 * 8;
            MVP_REQUIRE(grid > 0, "det conv: persistent grid");
            const dim3 gp((unsigned)grid), tp(256);
            auto go = [&](auto kern) { hipLaunchKernelGGL(kern, gp, tp, 0, s, p); };
            auto by_bn = [&](auto ks_tag, auto st_tag) {
                constexpr int K = decltype(ks_tag)::value, T = decltype(st_tag)::value;
                if (bn == 192) go(det_conv1x1_pers_kernel<192, 1, 3, K, T>);
                else if (bn == 128) go(det_conv1x1_pers_kernel<128, 1, 3, K, T>);
                else if (bn == 96) go(det_conv1x1_pers_kernel<96, 2, 3, K, T>);
                else if (bn == 64) go(det_conv1x1_pers_kernel<64, 1, 3, K, T>);
                else go(det_conv1x1_pers_kernel<32, 2, 3, K, T>);
            };
            if (ks == 1) by_bn(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
            else if (stride == 1) by_bn(std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{});
            else by_bn(std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{});
            MVP_HIP(hipGetLastError());
            return;
        }
    }
    const dim3 g((unsigned)blocks), t(256);
#define MVP_DET_CONV_BN(KS, S)                                                                         \
    do {                                                                                              \
        if (bn == 192)                                                                                \
            hipLaunchKernelGGL((det_conv_gemm_kernel<192, KS, S, 2, 3, 1>), g, t, 0, s, p);          \
        else if (bn == 128)                                                                           \
            hipLaunchKernelGGL((det_conv_gemm_kernel<128, KS, S, 2, 3, 1>), g, t, 0, s, p);          \
        else if (bn == 96)                                                                            \
            hipLaunchKernelGGL((det_conv_gemm_kernel<96, KS, S, 2, 3, 1>), g, t, 0, s, p);           \
        else if (bn == 64)                                                                            \
            hipLaunchKernelGGL((det_conv_gemm_kernel<64, KS, S, 2, 3, 1>), g, t, 0, s, p);           \
        else                                                                                          \
            hipLaunchKernelGGL((det_conv_gemm_kernel<32, KS, S, 2, 3, 1>), g, t, 0, s, p);           \
    } while (0)
    if (ks == 1)
        MVP_DET_CONV_BN(1, 1);
    else if (stride == 1)
        MVP_DET_CONV_BN(3, 1);
    else
        MVP_DET_CONV_BN(3, 2);
#undef MVP_DET_CONV_BN
    MVP_HIP(hipGetLastError());
}

template <int C, int TH, int TW>
void launch_dwpw_t(const DwPwParams& p, int n, hipStream_t s) {
    using G = DwPwCfg<C, TH, TW>;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)dwpw_kernel<C, TH, TW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    G::LDS));
        attr = true;
    }
    const int tiles = ((p.H + G::TH - 1) / G::TH) * p.tiles_w;
    hipLaunchKernelGGL((dwpw_kernel<C, TH, TW>), dim3((unsigned)tiles, (unsigned)n), dim3(512), G::LDS, s, p);
}

void launch_det_dwpw(const uint16_t* x, int xs, const float* dw_w, const float* dw_b, const uint16_t* wimg,
                     const float* pw_b, const uint16_t* res, int rs, uint16_t* y, int ys, int n, int H, int W, int C,
                     int N, int act_dw, int act_pw, hipStream_t s) {
    MVP_REQUIRE(det_dwpw_supported(C) && det_cout_pad(N) == C && xs % 8 == 0 && ys % 4 == 0 && (!res || rs % 4 == 0),
                "dwpw: C=%d cout=%d strides %d/%d", C, N, xs, ys);
    if (n == 0) return;
    MVP_REQUIRE(n < 65536 && (long)H * W < (1L << 26), "dwpw: grid too large");
    constexpr int TW = 16;
    DwPwParams p{x, dw_w, dw_b, wimg, pw_b, res, y, H, W, N, xs, ys, rs, act_dw, act_pw, (W + TW - 1) / TW};
    // 4 x 16 tiles: 36-44 KB of LDS, 3 workgroups per CU (8 x 16 tiles: 2 per CU, 83.5 vs 82.0 ms
    // per 512-frame forward same-box, gpurun_out/r06g)
    if (C == 64) launch_dwpw_t<64, 4, TW>(p, n, s);
    else launch_dwpw_t<96, 4, TW>(p, n, s);
    MVP_HIP(hipGetLastError());
}

// Measured per block, 512 frames (gpurun_out/detbd2, detbd3): 64 channels on 160x160 1.93 ms fused
// (4 x 16 tiles) vs 2.73 for dw5 + GEMM; 96 on 80x80 0.90 vs 1.20 (with the identity); with 8 x 8
// tiles 192 on 40x40 1.00 vs 0.68 and 384 on 20x20 1.12 vs 0.38 — the tile re-reads the whole
// C x C weight matrix and too few tiles hide the serial phases — so only 64 and 96 are fused.
bool det_dwpw_supported(int C) { return C == 64 || C == 96; }

void launch_det_ca(uint16_t* x, int xs, int n, int HW, int C, const float* wt, const float* b, float* scratch,
                   hipStream_t s, bool scale_pass) {
    static_assert(kCaSplit == 16, "det_ca_scales (det.h)");
    MVP_REQUIRE(C % 8 == 0 && C / 8 <= 256 && xs % 8 == 0, "ca: C=%d", C);
    const int rows = 256 / (C / 8);
    const size_t lds = (size_t)rows * C * sizeof(float);
    MVP_REQUIRE(lds <= 64 * 1024, "ca: C=%d needs too much LDS", C);
    if (n == 0) return;
    float* part = scratch;                              // [n][kCaSplit][C]
    float* sc = scratch + (size_t)n * kCaSplit * C;     // [n][C]
    CaParams p{x, wt, b, part, sc, HW, C, xs};
    hipLaunchKernelGGL(ca_pool_kernel, dim3(kCaSplit, (unsigned)n), dim3(256), lds, s, p);
    MVP_HIP(hipGetLastError());
    hipLaunchKernelGGL(ca_fc_kernel, dim3((unsigned)((C + 63) / 64), (unsigned)n), dim3(64), (size_t)C * sizeof(float),
                       s, p);
    MVP_HIP(hipGetLastError());
    if (!scale_pass) return;  // folded into the consumer conv (DetConvFold::ca)
    const long work = (long)HW * (C / 8);
    hipLaunchKernelGGL(ca_scale_kernel, dim3((unsigned)((work + 255) / 256), (unsigned)n), dim3(256), 0, s, x, sc, HW,
                       C, xs);
    MVP_HIP(hipGetLastError());
}

void launch_det_spp(uint16_t* buf, int xs, int n, int H, int W, int C, hipStream_t s) {
    MVP_REQUIRE(C % 8 == 0 && xs >= 4 * C && xs % 8 == 0, "spp: C=%d stride=%d", C, xs);
    // two planes of G 16-B chunks per pixel in LDS: with G = 4, H * W <= 1024 (20 x 20 = 400 at the
    // model's 640; 1,024 = the stride-32 plane of a 1,024 x 1,024 input); larger planes or
    // channel counts not a multiple of 32 take G = 1 (H * W <= 2048)
    const int G = (C % 32 == 0 && H * W <= 1024) ? 4 : 1;
    const size_t lds = (size_t)2 * H * W * G * sizeof(uint4);
    MVP_REQUIRE(lds <= 64 * 1024, "spp: %dx%d plane too large (H * W <= 2048)", H, W);
    if (n == 0) return;
    if (G == 4)
        hipLaunchKernelGGL(spp_kernel<4>, dim3((unsigned)(C / 32), (unsigned)n), dim3(256), lds, s, buf, H, W, C, xs);
    else
        hipLaunchKernelGGL(spp_kernel<1>, dim3((unsigned)(C / 8), (unsigned)n), dim3(256), lds, s, buf, H, W, C, xs);
    MVP_HIP(hipGetLastError());
}

void launch_det_up2(const uint16_t* x, int xs, uint16_t* y, int ys, int n, int H, int W, int C, hipStream_t s) {
    MVP_REQUIRE(C % 8 == 0 && xs % 8 == 0 && ys % 8 == 0, "up2: C=%d", C);
    const long work = (long)4 * H * W * (C / 8);
    if (n == 0 || work == 0) return;
    hipLaunchKernelGGL(up2_kernel, dim3((unsigned)((work + 255) / 256), (unsigned)n), dim3(256), 0, s, x, xs, y, ys, H,
                       W, C);
    MVP_HIP(hipGetLastError());
}

void launch_det_head(const uint16_t* x, int xs, int F, const float* w, const float* b, float* cand, int n, int H, int W,
                     int stride, int size, int n_priors, int prior0, hipStream_t s) {
    MVP_REQUIRE(F % 8 == 0 && xs >= 2 * F && prior0 + H * W <= n_priors, "det head: shape");
    HeadParams p{x, w, b, cand, H, W, F, xs, stride, size, n_priors, prior0};
    if (n == 0) return;
    const dim3 grid((unsigned)((H * W + 255) / 256), (unsigned)n);
    const char* e = getenv("MVPOSE_DET_HEAD_DIRECT");  // tests: 1 = one lane per pixel from HBM
    if (F % kHeadKC == 0 && !(e && e[0] == '1'))
        hipLaunchKernelGGL(det_head_staged_kernel, grid, dim3(256),
                           (size_t)((5 * F + 3) & ~3) * sizeof(float) + 256 * 9 * sizeof(uint4), s, p);
    else
        hipLaunchKernelGGL(det_head_kernel, grid, dim3(256), (size_t)5 * F * sizeof(float), s, p);
    MVP_HIP(hipGetLastError());
}

void launch_det_select(const float* cand, int n, int n_priors, float score_thr, float fx, float fy, float* best,
                       hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(det_select_kernel, dim3((unsigned)n), dim3(256), 0, s, cand, n_priors, score_thr, fx, fy, best);
    MVP_HIP(hipGetLastError());
}

}  // namespace mvp

extern "C" int mvp_det_letterbox(const uint8_t* frames, int n, int h, int w, int size, const float* mean3,
                                 const float* std3, void* out, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n >= 0 && h > 0 && w > 0 && size > 0 && mean3 && std3, "mvp_det_letterbox: bad arguments");
    MVP_REQUIRE(n == 0 || (frames && out), "mvp_det_letterbox: NULL buffer");
    mvp::launch_det_letterbox(frames, n, h, w, size, mean3, std3, out, reinterpret_cast<hipStream_t>(stream));
    MVP_ABI_END
}

extern "C" int mvp_det_nms(const float* cand, int n, int n_priors, const int* level_off, int n_levels, int nms_pre,
                           float score_thr, float iou_thr, int max_det, float fx, float fy, float* dets, int* counts,
                           void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n >= 0 && n_levels >= 1 && n_levels <= 3 && level_off, "mvp_det_nms: bad levels");
    MVP_REQUIRE(nms_pre >= 1 && nms_pre <= 1024 && max_det >= 1, "mvp_det_nms: nms_pre must be in [1, 1024]");
    MVP_REQUIRE(level_off[0] == 0 && level_off[n_levels] == n_priors, "mvp_det_nms: level offsets");
    int offs[4];
    for (int l = 0; l <= n_levels; l++) offs[l] = level_off[l];
    for (int l = 0; l < n_levels; l++)
        MVP_REQUIRE(offs[l + 1] > offs[l] && offs[l + 1] - offs[l] <= mvp::kNmsCap, "mvp_det_nms: level %d has %d priors",
                    l, offs[l + 1] - offs[l]);
    if (n == 0) return MVP_OK;
    MVP_REQUIRE(cand && dets && counts, "mvp_det_nms: NULL buffer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int* d_off = nullptr;
    MVP_HIP(hipMallocAsync((void**)&d_off, sizeof(offs), s));
    MVP_HIP(hipMemcpyAsync(d_off, offs, sizeof(int) * (n_levels + 1), hipMemcpyHostToDevice, s));
    const size_t lds = (size_t)mvp::kNmsCap * sizeof(unsigned long long);
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)mvp::det_nms_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
        attr = true;
    }
    hipLaunchKernelGGL(mvp::det_nms_kernel, dim3((unsigned)n), dim3(1024), lds, s, cand, n_priors, d_off, n_levels,
                       nms_pre, score_thr, iou_thr, max_det, fx, fy, dets, counts);
    MVP_HIP(hipGetLastError());
    MVP_HIP(hipFreeAsync(d_off, s));
    MVP_ABI_END
}
