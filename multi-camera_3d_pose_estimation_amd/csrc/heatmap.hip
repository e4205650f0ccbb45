// 2D-stage kernels around the backbone (gfx950):
//
//  * preprocess_kernel — mmpose TopdownAffine + PoseDataPreprocessor for the
//    whole-frame bbox (reference mmpose_pose_estimation.py:253, bboxes=None
//    fallback at :246-250): cv2.warpAffine(INTER_LINEAR) of the uint8 frame to
//    256x192 with OpenCV's fixed-point mapping (AB_BITS 10, INTER_BITS 5) and
//    integer bilinear weights, then bgr_to_rgb + (x - mean) / std in f32 ->
//    bf16 NHWC with a zero 4th channel; the horizontally flipped crop for the
//    flip test is written in the same pass.
//  * decode_kernel — flip-test average (flip_mode='heatmap', shift_heatmap),
//    MSRAHeatmap decode (first-occurrence argmax, val<=0 -> -1, +-0.25 sign
//    refinement inside 1<px<W-1, 1<py<H-1, x4) and the keypoint restore to image
//    pixels (TopdownPoseEstimator.add_pred_to_datasample).  One wave per map.
//  * moments_kernel — revert_heatmap (cv2.warpAffine of the 64x48 map to the
//    full image, float weights) fused with PoseEstimator.get_heatmap_means_cov
//    (mmpose_pose_estimation.py:163-215): h<0.01 -> 0, normalised mean and
//    covariance.  The 17 x H x W reverted heatmap is never written: each lane
//    evaluates the warp for its image pixels from the LDS-resident map and
//    accumulates fp64 raw moments.
#include <algorithm>
#include <cstdlib>

#include "mvp_common.h"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}

// ---------------------------------------------------------------- preprocess
struct PreParams {
    const uint8_t* __restrict__ frames;
    const double* __restrict__ minv;  // [n][6] crop -> image (warpAffine's inverted map)
    uint16_t* __restrict__ out;
    int n, H, W, oh, ow, swap_rb, flip;
    float mean[3], stdv[3];
};

// one grid row per crop, 32-bit in-crop index (the flat 64-bit index's three divisions
// per pixel made the kernel VALU-bound)
__global__ __launch_bounds__(kBlock) void preprocess_kernel(PreParams p) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const int n = blockIdx.y;
    if (i >= p.oh * p.ow) return;
    const int y = (int)((unsigned)i / (unsigned)p.ow), x = i - y * p.ow;
    const double* M = p.minv + 6 * n;
    // WarpAffineInvoker: X0/Y0 per row, adelta/bdelta per column (cvRound = rint)
    const int X0 = (int)rint((M[1] * y + M[2]) * 1024.0) + 16;
    const int Y0 = (int)rint((M[4] * y + M[5]) * 1024.0) + 16;
    const int X = (X0 + (int)rint(M[0] * x * 1024.0)) >> 5;
    const int Y = (Y0 + (int)rint(M[3] * x * 1024.0)) >> 5;
    const int sx = X >> 5, sy = Y >> 5, tx = X & 31, ty = Y & 31;
    const int w[4] = {(32 - ty) * (32 - tx) * 32, (32 - ty) * tx * 32, ty * (32 - tx) * 32, ty * tx * 32};
    int acc[3] = {0, 0, 0};
    const uint8_t* img = p.frames + (size_t)n * p.H * p.W * 3;
    // each source row's two pixels are 6 contiguous bytes: away from the right edge (and with
    // 4-byte-aligned rows) 3 dword loads and two byte alignments instead of 6 byte loads (round 6);
    // the integer sums are exact, so the order of the terms does not matter
    const bool fast = (p.W & 3) == 0 && sx >= 0 && sx + 3 < p.W;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int yy = sy + r;
        if (yy < 0 || yy >= p.H) continue;
        const uint8_t* row = img + (size_t)yy * p.W * 3;
        if (fast) {
            const int b0 = 3 * sx, sh = b0 & 3;
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(row + (b0 & ~3));
            const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, sh), d1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
            const int wl = w[2 * r], wr = w[2 * r + 1];
            acc[0] += (int)(d0 & 0xff) * wl + (int)((d0 >> 24) & 0xff) * wr;
            acc[1] += (int)((d0 >> 8) & 0xff) * wl + (int)(d1 & 0xff) * wr;
            acc[2] += (int)((d0 >> 16) & 0xff) * wl + (int)((d1 >> 8) & 0xff) * wr;
            continue;
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int xx = sx + h;
            if (xx >= 0 && xx < p.W) {
                const uint8_t* px = row + (size_t)xx * 3;
                acc[0] += px[0] * w[2 * r + h];
                acc[1] += px[1] * w[2 * r + h];
                acc[2] += px[2] * w[2 * r + h];
            }
        }
    }
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        int u = (acc[c] + (1 << 14)) >> 15;
        u = u < 0 ? 0 : (u > 255 ? 255 : u);
        v[c] = (float)u;
    }
    uint16_t o[4];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const float src = p.swap_rb ? v[2 - c] : v[c];
        o[c] = f32_to_bf16(__fdiv_rn(src - p.mean[c], p.stdv[c]));
    }
    o[3] = 0;
    uint2 packed;
    packed.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
    packed.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
    *reinterpret_cast<uint2*>(p.out + (((size_t)n * p.oh + y) * p.ow + x) * 4) = packed;
    if (p.flip)
        *reinterpret_cast<uint2*>(p.out + (((size_t)(n + p.n) * p.oh + y) * p.ow + (p.ow - 1 - x)) * 4) = packed;
}

// ---------------------------------------------------------------- decode
struct DecodeParams {
    const float* __restrict__ hm;
    const float* __restrict__ hmf;  // nullable: flipped-input heatmaps
    const float* __restrict__ cs;   // [N][4] center x, y, scale w, h
    float* __restrict__ avg;        // nullable
    float* __restrict__ kpts;
    float* __restrict__ scores;
    int* __restrict__ amax;
    float* __restrict__ tkv;        // nullable: [N/V][K][3][V] (reference kpts_2d layout)
    int N, K, H, W, shift, V;
    int flip_idx[32];
    double in_w, in_h;
};

// value of the (flip-averaged) map at (y, x): (h + shifted flipped h) * 0.5 in f32
__device__ __forceinline__ float avg_at(const DecodeParams& p, const float* h, const float* hf, int y, int x) {
    const float a = h[y * p.W + x];
    if (!hf) return a;
    int xs = x;
    if (p.shift && x >= 1) xs = x - 1;  // heatmaps[..., 1:] = heatmaps[..., :-1]
    const float b = hf[y * p.W + (p.W - 1 - xs)];
    return __fmul_rn(__fadd_rn(a, b), 0.5f);
}

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
    // np.argmax: first occurrence of the max; NaN counts as the max (first NaN wins)
    const bool vn = isnan(v), bn = isnan(bv);
    if (bn) return vn && i < bi;
    if (vn) return true;
    return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(kBlock) void decode_kernel(DecodeParams p) {
    const int lane = threadIdx.x & 63;
    const long map = (long)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (map >= (long)p.N * p.K) return;
    const int n = map / p.K, k = map % p.K;
    const int HW = p.H * p.W;
    const float* h = p.hm + map * HW;
    const float* hf = p.hmf ? p.hmf + ((long)n * p.K + p.flip_idx[k]) * HW : nullptr;
    float* av = p.avg ? p.avg + map * HW : nullptr;
    float bv = 0.f;
    int bi = 0x7fffffff;
    if ((p.W & 3) == 0 && (HW & 255) == 0) {
        // 4 consecutive cells of one row per lane (16-B loads / stores of the map and the
        // average, 4 mirrored loads of the flipped map): four times the bytes in flight of
        // one cell per lane, which left the kernel latency-bound
        int i0 = lane * 4, y = i0 / p.W, x = i0 - y * p.W;
        for (; i0 < HW; i0 += 256) {
            const float4 a4 = *reinterpret_cast<const float4*>(h + i0);
            float v[4] = {a4.x, a4.y, a4.z, a4.w};
            if (hf) {
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    int xs = x + e;
                    if (p.shift && xs >= 1) xs -= 1;  // heatmaps[..., 1:] = heatmaps[..., :-1]
                    v[e] = __fmul_rn(__fadd_rn(v[e], hf[y * p.W + (p.W - 1 - xs)]), 0.5f);
                }
            }
            if (av) *reinterpret_cast<float4*>(av + i0) = float4{v[0], v[1], v[2], v[3]};
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (bi == 0x7fffffff || better(v[e], i0 + e, bv, bi)) {
                    bv = v[e];
                    bi = i0 + e;
                }
            x += 256;
            while (x >= p.W) {
                x -= p.W;
                y++;
            }
        }
    } else {
        int y = lane / p.W, x = lane - y * p.W;  // (y, x) of i, stepped without divisions
        for (int i = lane; i < HW; i += 64) {
            const float v = avg_at(p, h, hf, y, x);
            x += 64;
            while (x >= p.W) {
                x -= p.W;
                y++;
            }
            if (av) av[i] = v;
            if (bi == 0x7fffffff || better(v, i, bv, bi)) {
                bv = v;
                bi = i;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off);
        const int oi = __shfl_xor(bi, off);
        if (oi != 0x7fffffff && (bi == 0x7fffffff || better(ov, oi, bv, bi))) {
            bv = ov;
            bi = oi;
        }
    }
    if (lane != 0) return;
    const int py = bi / p.W, px = bi - (bi / p.W) * p.W;
    float kx = (float)px, ky = (float)py;
    if (!(bv > 0.f)) {  // locs[vals <= 0.] = -1 (NaN > 0 is false but NaN <= 0 is false too)
        if (!isnan(bv)) {
            kx = -1.f;
            ky = -1.f;
        }
    }
    const int ipx = (int)kx, ipy = (int)ky;
    if (1 < ipx && ipx < p.W - 1 && 1 < ipy && ipy < p.H - 1) {
        const float dx = __fsub_rn(avg_at(p, h, hf, ipy, ipx + 1), avg_at(p, h, hf, ipy, ipx - 1));
        const float dy = __fsub_rn(avg_at(p, h, hf, ipy + 1, ipx), avg_at(p, h, hf, ipy - 1, ipx));
        const float sgx = dx > 0.f ? 1.f : (dx < 0.f ? -1.f : (isnan(dx) ? dx : 0.f));
        const float sgy = dy > 0.f ? 1.f : (dy < 0.f ? -1.f : (isnan(dy) ? dy : 0.f));
        kx = __fadd_rn(kx, __fmul_rn(sgx, 0.25f));
        ky = __fadd_rn(ky, __fmul_rn(sgy, 0.25f));
    }
    // * scale_factor (input_size / heatmap_size, f32)
    kx = __fmul_rn(kx, (float)(p.in_w / p.W));
    ky = __fmul_rn(ky, (float)(p.in_h / p.H));
    // keypoints / input_size * input_scale + input_center - 0.5 * input_scale (f64, stored f32)
    const float* cs = p.cs + 4 * n;
    const double ox = (double)kx / p.in_w * (double)cs[2] + (double)cs[0] - 0.5 * (double)cs[2];
    const double oy = (double)ky / p.in_h * (double)cs[3] + (double)cs[1] - 0.5 * (double)cs[3];
    p.kpts[2 * map + 0] = (float)ox;
    p.kpts[2 * map + 1] = (float)oy;
    p.scores[map] = bv;
    if (p.amax) p.amax[map] = bi;
    if (p.tkv) {  // crops ordered (t, v): pose_estimation.py:135 stacks [x, y, score] per camera on the last axis
        const int t = n / p.V, v = n - (n / p.V) * p.V;
        float* o = p.tkv + (((long)t * p.K + k) * 3) * p.V + v;
        o[0] = (float)ox;
        o[p.V] = (float)oy;
        o[2 * p.V] = bv;
    }
}

// ---------------------------------------------------------------- moments
struct MomParams {
    const float* __restrict__ hm;     // [N][K][h][w] (flip-averaged)
    const double* __restrict__ minv;  // [N][6] image -> heatmap (warpAffine's inverted map)
    double* __restrict__ out;         // [N][K][6]
    int N, K, h, w, img_h, img_w;
    float thr;
    int separable;  // host-verified: source column depends on x only, source row on y only
                    // (2: the separable path without the per-run closed forms)
    const int* __restrict__ sep;  // nullable: per-crop flags (mvp_bbox_geometry); a crop whose flag
                                  // is 0 takes the general path, the others `separable`
    int jpb;        // joints per workgroup: the warp tables depend on the crop only, so a
                    // workgroup builds them once and reuses them for jpb maps of its crop
    int mixcf;      // separable path: mixed columns in closed form with a per-row prefix table
};

constexpr int kMomMaxLds = 64 * 1024;  // dynamic LDS budget: map + 2 int column tables
constexpr int kMomMaxLdsCf = 96 * 1024;  // ... + the per-row prefix table of the mixed-column closed forms
constexpr int kMomBlock = 320;         // 5 waves x 4 columns per lane = 1280: every lane busy on 1280-wide frames
constexpr int kMomCols = 4;            // image columns per lane (separable path)
constexpr int kMomJointsPerBlock = 17;  // maps per workgroup sharing one set of warp tables (all of a
                                        // COCO crop: 8680-8717 -> 8823-8832 frames/s in the bench vs 1)
static_assert(kMomBlock % 64 == 0 && kMomCols % 2 == 0, "whole waves (per-wave reduction slots), packed column pairs");

// One workgroup per (crop, group of jpb joints); the column / row / run tables are
// built once per workgroup, then the maps of its joints are processed in turn.  The fixed-point warp of an image pixel
// (OpenCV WarpAffineInvoker) is X = (X0(y) + adelta(x)) >> 5, Y = (Y0(y) + bdelta(x)) >> 5.
// Separable path (axis-aligned crops, the only ones the pipeline makes): each
// lane owns image columns (source column ix and weight fx fixed), walks the rows,
// keeps the 4 taps in registers while the source row iy stays the same (~33
// image rows per heatmap row), and accumulates per column S, S·y, S·y² in fp64;
// x-moments are applied per column at the end.  Rows / columns whose taps are
// all below thr·(1-1e-6) contribute exact zeros and are skipped (bounding box
// of active heatmap cells).
__global__ __launch_bounds__(kMomBlock) void moments_kernel(MomParams p) {
    extern __shared__ __attribute__((aligned(16))) float mom_lds[];
    float* shm = mom_lds;
    int* sad = reinterpret_cast<int*>(mom_lds + ((p.h * p.w + 3) & ~3));
    int* sbd = sad + p.img_w;
    int* riy = sbd + p.img_w;  // separable path: per image row source row / weight index
    // separable path, per run of image rows sharing source row iy = r - 1 (r = 0 .. h):
    // first / one-past-last image row and the run's weight sums (mom_run_layout)
    int* rstart = riy + ((p.img_h + 2) & ~1);
    int* rend = rstart + ((p.h + 2) & ~1);  // even int counts keep rsum 8-B aligned
    double* rsum = reinterpret_cast<double*>(rend + ((p.h + 2) & ~1));
    // mixed-column closed forms: per image row y, the run-inclusive prefix over the rows of
    // y's run up to y of gy, fy, gy·yr, fy·yr, gy·yr², fy·yr² (yr = row - run start)
    double* rpre = rsum + 6 * (p.h + 1);
    __shared__ double red[6][kMomBlock / 64];
    __shared__ int bbox[4];
    const int groups = (p.K + p.jpb - 1) / p.jpb;
    const int n = blockIdx.x / groups;
    const int k0 = (blockIdx.x - n * groups) * p.jpb, k1 = min(p.K, k0 + p.jpb);
    const double* M = p.minv + 6 * n;
    const int separable = (p.sep && !p.sep[n]) ? 0 : p.separable;
    for (int x = threadIdx.x; x < p.img_w; x += kMomBlock) {
        sad[x] = (int)rint(M[0] * x * 1024.0);
        sbd[x] = (int)rint(M[3] * x * 1024.0);
    }
    __syncthreads();
    const double cx = 0.5 * p.img_w, cy = 0.5 * p.img_h;  // centred coordinates (cancellation)
    if (separable) {
        // Row table: source row iy and weight index fq of every image row (uniform per row).
        // packed (iy + 4096) << 5 | fq, one word per row
        for (int r = threadIdx.x; r <= p.h; r += kMomBlock) {
            rstart[r] = p.img_h;
            rend[r] = 0;
        }
        __syncthreads();
        for (int y = threadIdx.x; y < p.img_h; y += kMomBlock) {
            const int Yq = ((int)rint((M[4] * y + M[5]) * 1024.0) + 16 + sbd[0]) >> 5;
            const int iy = Yq >> 5;
            riy[y] = ((iy + 4096) << 5) | (Yq & 31);
            if (iy >= -1 && iy < p.h) {  // rows of other runs read no map row: zero
                atomicMin(&rstart[iy + 1], y);
                atomicMax(&rend[iy + 1], y + 1);
            }
        }
        __syncthreads();
        // Per run (the affine row map is monotone, so a run is contiguous): sums over its
        // rows of gy, fy, gy·yr, fy·yr, gy·yr², fy·yr² (yr = row - run start), exact in fp64.
        // A column whose 4 taps are all >= thr·(1+2e-6) has every pixel of the run above
        // the threshold (a bilinear value is a convex combination of its taps): its run
        // sums are a·G + b·F in closed form.  Taps all < thr·(1-2e-6): all zero.  Only
        // the remaining ("mixed") columns walk the run's rows.
        for (int r = threadIdx.x; r <= p.h; r += kMomBlock) {
            double g0 = 0, f0 = 0, g1 = 0, f1 = 0, g2 = 0, f2 = 0;
            for (int y = rstart[r]; y < rend[r]; y++) {
                const double fy = (double)(riy[y] & 31) * (1.0 / 32.0), gy = 1.0 - fy;
                const double yr = y - rstart[r];
                g0 += gy;
                f0 += fy;
                g1 += gy * yr;
                f1 += fy * yr;
                g2 += gy * yr * yr;
                f2 += fy * yr * yr;
                if (p.mixcf) {
                    double* pr = rpre + 6 * y;
                    pr[0] = g0;
                    pr[1] = f0;
                    pr[2] = g1;
                    pr[3] = f1;
                    pr[4] = g2;
                    pr[5] = f2;
                }
            }
            // folded with the run's centred offset y0c = start - cy: a closed-form column
            // adds a·q[0] + b·q[1] to S, a·q[2] + b·q[3] to Sy and a·q[4] + b·q[5] to Syy
            const double y0c = rstart[r] - cy;
            double* q = rsum + 6 * r;
            q[0] = g0;
            q[1] = f0;
            q[2] = y0c * g0 + g1;
            q[3] = y0c * f0 + f1;
            q[4] = y0c * y0c * g0 + 2.0 * y0c * g1 + g2;
            q[5] = y0c * y0c * f0 + 2.0 * y0c * f1 + f2;
        }
        __syncthreads();
    }
    const float thr_lo = p.thr * (1.f - 1e-6f);
    for (int kj = k0; kj < k1; kj++) {
        const long map = (long)n * p.K + kj;
        const float* src = p.hm + map * p.h * p.w;
        if (threadIdx.x == 0) {  // every thread read the previous map's bbox before its reduction barrier
            bbox[0] = p.w;
            bbox[1] = -1;
            bbox[2] = p.h;
            bbox[3] = -1;
        }
        __syncthreads();
        int c0 = p.w, c1 = -1, r0 = p.h, r1 = -1;
        for (int i = threadIdx.x; i < p.h * p.w; i += kMomBlock) {
            const float v = src[i];
            shm[i] = v;
            if (!(v < thr_lo)) {  // active (or NaN)
                const int r = i / p.w, c = i - (i / p.w) * p.w;
                c0 = min(c0, c);
                c1 = max(c1, c);
                r0 = min(r0, r);
                r1 = max(r1, r);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            c0 = min(c0, __shfl_xor(c0, off));
            c1 = max(c1, __shfl_xor(c1, off));
            r0 = min(r0, __shfl_xor(r0, off));
            r1 = max(r1, __shfl_xor(r1, off));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&bbox[0], c0);
            atomicMax(&bbox[1], c1);
            atomicMin(&bbox[2], r0);
            atomicMax(&bbox[3], r1);
        }
        __syncthreads();
        c0 = bbox[0];
        c1 = bbox[1];
        r0 = bbox[2];
        r1 = bbox[3];
        double t[6] = {0, 0, 0, 0, 0, 0};
        if (c1 >= 0) {
            if (separable) {
                // Lanes own column pairs (packed f32 math).  Per run, a column's two
                // x-interpolated source rows a = v00 gx + v01 fx and b = v10 gx + v11 fx are
                // formed once; the pixel value is OpenCV's bilinear remap value (its fixed-point
                // coordinates and 1/32 weights exactly) evaluated as gy a + fy b: within ~2 f32
                // ulps of OpenCV's operation order ((v00 w0 + v01 w1) + v10 w2) + v11 w3 — far
                // inside the reference's own f32 moment arithmetic (mmpose_pose_estimation.py:163-215).
                // Mixed columns accumulate S, S*yr, S*yr^2 over the run's rows in f32, flushed
                // to fp64 with the run's offset.
                typedef float f2 __attribute__((ext_vector_type(2)));
                constexpr int NP = kMomCols / 2;
                const int X0 = (int)rint((M[1] * 0 + M[2]) * 1024.0) + 16;
                const float thr_hi = p.thr * (1.f + 2e-6f), thr_lo2 = p.thr * (1.f - 2e-6f);
                const bool closed = separable != 2;  // 2: walk every column (diagnostics / tests)
                for (int xb = threadIdx.x; xb < p.img_w; xb += kMomBlock * kMomCols) {
#pragma clang fp contract(off)
                    int ix[kMomCols];
                    bool on[kMomCols];
                    float gx[kMomCols], fx[kMomCols];
                    bool any = false;
#pragma unroll
                    for (int j = 0; j < kMomCols; j++) {
                        const int x = xb + j * kMomBlock;
                        const int X = (x < p.img_w) ? ((X0 + sad[x]) >> 5) : 0;
                        ix[j] = X >> 5;
                        const float f = (float)(X & 31) * (1.f / 32.f);
                        fx[j] = f;
                        gx[j] = 1.f - f;
                        on[j] = x < p.img_w && ix[j] + 1 >= c0 && ix[j] <= c1;
                        any |= on[j];
                    }
                    double S[kMomCols], Sy[kMomCols], Syy[kMomCols];
#pragma unroll
                    for (int j = 0; j < kMomCols; j++) S[j] = Sy[j] = Syy[j] = 0.0;
                    if (__any(any)) {
                        const f2 thr2 = f2{p.thr, p.thr};
                        for (int r = max(r0, 0); r <= min(r1 + 1, p.h); r++) {  // iy = r - 1 in [r0 - 1, r1]
                            const int ys = rstart[r], ye = rend[r];
                            if (ys >= ye) continue;
                            const int iy = r - 1;
                            const bool ry0 = iy >= 0, ry1 = iy + 1 < p.h;
                            const double* q = rsum + 6 * r;
                            const double y0c = ys - cy;
                            f2 ra[NP], rb[NP];
                            bool mixed = false;
#pragma unroll
                            for (int j = 0; j < kMomCols; j++) {
                                const bool cx0 = ix[j] >= 0 && ix[j] < p.w, cx1 = ix[j] + 1 >= 0 && ix[j] + 1 < p.w;
                                const float v00 = (on[j] && ry0 && cx0) ? shm[iy * p.w + ix[j]] : 0.f;
                                const float v01 = (on[j] && ry0 && cx1) ? shm[iy * p.w + ix[j] + 1] : 0.f;
                                const float v10 = (on[j] && ry1 && cx0) ? shm[(iy + 1) * p.w + ix[j]] : 0.f;
                                const float v11 = (on[j] && ry1 && cx1) ? shm[(iy + 1) * p.w + ix[j] + 1] : 0.f;
                                const float a = __builtin_fmaf(v01, fx[j], v00 * gx[j]);
                                const float b = __builtin_fmaf(v11, fx[j], v10 * gx[j]);
                                const bool full = closed && v00 >= thr_hi && v01 >= thr_hi && v10 >= thr_hi && v11 >= thr_hi;
                                const bool empty = closed && v00 < thr_lo2 && v01 < thr_lo2 && v10 < thr_lo2 && v11 < thr_lo2;
                                if (full) {
                                    const double da = a, db = b;
                                    S[j] = fma(da, q[0], fma(db, q[1], S[j]));
                                    Sy[j] = fma(da, q[2], fma(db, q[3], Sy[j]));
                                    Syy[j] = fma(da, q[4], fma(db, q[5], Syy[j]));
                                }
                                bool walk = !full && !empty;
                                // Mixed column in closed form: the walk's pixel value
                                // v(y) = fy·b + gy·a (f32, gy·a rounded first) is linear in fy,
                                // and fy grows with y inside a run, so its rows at or above thr
                                // form a prefix or a suffix of the run.  When |b - a| / 32 (the
                                // least change of the exact value between rows) exceeds 4 ulps of
                                // max(|a|, |b|) — twice the evaluation's rounding — the computed
                                // v is monotone too, so the exact f32 decisions of a binary search
                                // find the cut, and the above-threshold rows' sums come from the
                                // run's prefix table: a·G + b·F in fp64 (the walk sums the same
                                // rows' f32 values in f32).  Otherwise the column walks.
                                if (walk && p.mixcf) {
                                    const float mag = fmaxf(fabsf(a), fabsf(b));
                                    if (fabsf(b - a) > mag * 1.6e-5f) {
                                        auto above = [&](int y) {
                                            const float fy = (float)(riy[y] & 31) * (1.f / 32.f), gy = 1.f - fy;
                                            return __builtin_fmaf(fy, b, gy * a) >= p.thr;
                                        };
                                        const bool d0 = above(ys), d1 = above(ye - 1);
                                        int u0 = ys, u1 = ys;  // above-threshold rows [u0, u1)
                                        if (d0 && d1) {
                                            u1 = ye;
                                        } else if (!d0 && d1) {
                                            int lo = ys, hi = ye - 1;
                                            while (hi - lo > 1) {
                                                const int mid = (lo + hi) >> 1;
                                                if (above(mid)) hi = mid;
                                                else lo = mid;
                                            }
                                            u0 = hi;
                                            u1 = ye;
                                        } else if (d0 && !d1) {
                                            int lo = ys, hi = ye - 1;
                                            while (hi - lo > 1) {
                                                const int mid = (lo + hi) >> 1;
                                                if (above(mid)) lo = mid;
                                                else hi = mid;
                                            }
                                            u1 = lo + 1;
                                        }
                                        if (u1 > u0) {
                                            const double* pe = rpre + 6 * (u1 - 1);
                                            double sg0 = pe[0], sf0 = pe[1], sg1 = pe[2], sf1 = pe[3], sg2 = pe[4],
                                                   sf2 = pe[5];
                                            if (u0 > ys) {
                                                const double* pb = rpre + 6 * (u0 - 1);
                                                sg0 -= pb[0];
                                                sf0 -= pb[1];
                                                sg1 -= pb[2];
                                                sf1 -= pb[3];
                                                sg2 -= pb[4];
                                                sf2 -= pb[5];
                                            }
                                            const double da = a, db = b;
                                            const double s0 = da * sg0 + db * sf0, s1 = da * sg1 + db * sf1,
                                                         s2 = da * sg2 + db * sf2;
                                            S[j] += s0;
                                            Sy[j] += y0c * s0 + s1;
                                            Syy[j] += y0c * y0c * s0 + 2.0 * y0c * s1 + s2;
                                        }
                                        walk = false;
                                    }
                                }
                                mixed |= walk;
                                ra[j / 2][j & 1] = walk ? a : 0.f;
                                rb[j / 2][j & 1] = walk ? b : 0.f;
                            }
                            if (!__any(mixed)) continue;  // every column of the wave done in closed form
                            f2 s32[NP], sy32[NP], syy32[NP];
#pragma unroll
                            for (int k = 0; k < NP; k++) s32[k] = sy32[k] = syy32[k] = f2{0.f, 0.f};
                            for (int y = ys; y < ye; y++) {
                                const int fq = riy[y] & 31;
                                const float fy = (float)fq * (1.f / 32.f), gy = 1.f - fy;
                                const float yr = (float)(y - ys);
                                const f2 yr2 = f2{yr, yr}, yrr2 = f2{yr * yr, yr * yr};
                                const f2 fy2 = f2{fy, fy}, gy2 = f2{gy, gy};
#pragma unroll
                                for (int k = 0; k < NP; k++) {
                                    const f2 v = __builtin_elementwise_fma(fy2, rb[k], gy2 * ra[k]);
                                    const f2 vs = f2{v.x >= thr2.x ? v.x : 0.f, v.y >= thr2.y ? v.y : 0.f};  // h[h < thr] = 0
                                    s32[k] = s32[k] + vs;
                                    sy32[k] = __builtin_elementwise_fma(vs, yr2, sy32[k]);
                                    syy32[k] = __builtin_elementwise_fma(vs, yrr2, syy32[k]);
                                }
                            }
#pragma unroll
                            for (int j = 0; j < kMomCols; j++) {
                                const double a = s32[j / 2][j & 1], b = sy32[j / 2][j & 1], c = syy32[j / 2][j & 1];
                                S[j] += a;
                                Sy[j] += y0c * a + b;
                                Syy[j] += y0c * y0c * a + 2.0 * y0c * b + c;
                            }
                        }
                    }
#pragma unroll
                    for (int j = 0; j < kMomCols; j++) {
                        const double xc = (double)(xb + j * kMomBlock) - cx;
                        t[0] += S[j];
                        t[1] = fma(xc, S[j], t[1]);
                        t[2] += Sy[j];
                        t[3] = fma(xc * xc, S[j], t[3]);
                        t[4] = fma(xc, Sy[j], t[4]);
                        t[5] += Syy[j];
                    }
                }
            } else {
                for (int y = 0; y < p.img_h; y++) {
                    const int X0 = (int)rint((M[1] * y + M[2]) * 1024.0) + 16;
                    const int Y0 = (int)rint((M[4] * y + M[5]) * 1024.0) + 16;
                    const double yc = y - cy;
                    for (int x = threadIdx.x; x < p.img_w; x += kMomBlock) {
                        const int X = (X0 + sad[x]) >> 5;
                        const int Y = (Y0 + sbd[x]) >> 5;
                        const int ix = X >> 5, iy = Y >> 5;
                        if (ix >= p.w || ix + 1 < 0 || iy >= p.h || iy + 1 < 0) continue;  // border value 0
                        const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
                        const float w0 = __fmul_rn(1.f - fy, 1.f - fx), w1 = __fmul_rn(1.f - fy, fx);
                        const float w2 = __fmul_rn(fy, 1.f - fx), w3 = __fmul_rn(fy, fx);
                        const bool x0 = ix >= 0, x1 = ix + 1 < p.w, y0 = iy >= 0, y1 = iy + 1 < p.h;
                        const float v0 = (x0 && y0) ? shm[iy * p.w + ix] : 0.f;
                        const float v1 = (x1 && y0) ? shm[iy * p.w + ix + 1] : 0.f;
                        const float v2 = (x0 && y1) ? shm[(iy + 1) * p.w + ix] : 0.f;
                        const float v3 = (x1 && y1) ? shm[(iy + 1) * p.w + ix + 1] : 0.f;
                        float v = __fmul_rn(v0, w0);
                        v = __fadd_rn(v, __fmul_rn(v1, w1));
                        v = __fadd_rn(v, __fmul_rn(v2, w2));
                        v = __fadd_rn(v, __fmul_rn(v3, w3));
                        if (!(v >= p.thr)) continue;
                        const double dv = v, xc = x - cx;
                        t[0] += dv;
                        t[1] += xc * dv;
                        t[2] += yc * dv;
                        t[3] += xc * xc * dv;
                        t[4] += xc * yc * dv;
                        t[5] += yc * yc * dv;
                    }
                }
            }
        }
        // t = {S, Sx, Sy, Sxx, Sxy, Syy}
#pragma unroll
        for (int q = 0; q < 6; q++) {
            double v = t[q];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            t[q] = v;
        }
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 6; q++) red[q][wv] = t[q];
        __syncthreads();
        if (threadIdx.x == 0) {
            double a[6];
#pragma unroll
            for (int q = 0; q < 6; q++) {
                a[q] = 0;
                for (int k = 0; k < kMomBlock / 64; k++) a[q] += red[q][k];
            }
            double* o = p.out + 6 * map;
            if (a[0] == 0.0) {
                for (int q = 0; q < 6; q++) o[q] = 0.0;
            } else {
                const double mxc = a[1] / a[0], myc = a[2] / a[0];
                const double vxx = a[3] / a[0] - mxc * mxc;
                const double vxy = a[4] / a[0] - mxc * myc;
                const double vyy = a[5] / a[0] - myc * myc;
                o[0] = mxc + cx;
                o[1] = myc + cy;
                o[2] = vxx;
                o[3] = vxy;
                o[4] = vxy;
                o[5] = vyy;
            }
        }
    }  // joints of this workgroup
}

// ---------------------------------------------------------------- revert only
// mmpose merge_data_samples' revert_heatmap (cv2.warpAffine INTER_LINEAR, BORDER_CONSTANT
// 0) of each crop's K flip-averaged maps to the full image: the values moments_kernel's
// general path thresholds, in OpenCV's fixed-point coordinates and operation order.
// Not on the hot path (moments fuse the revert); PoseEstimator.predict(return_full_heatmaps).
// Grid (ceil(img_w / 256), img_h, N); a thread computes one pixel's taps once for all K maps.
__global__ __launch_bounds__(kBlock) void revert_kernel(const float* __restrict__ hm, const double* __restrict__ minv,
                                                        float* __restrict__ out, int K, int h, int w, int img_h,
                                                        int img_w) {
    const int x = blockIdx.x * kBlock + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
    if (x >= img_w) return;
    const double* M = minv + 6 * n;
    const int X0 = (int)rint((M[1] * y + M[2]) * 1024.0) + 16;
    const int Y0 = (int)rint((M[4] * y + M[5]) * 1024.0) + 16;
    const int X = (X0 + (int)rint(M[0] * x * 1024.0)) >> 5;
    const int Y = (Y0 + (int)rint(M[3] * x * 1024.0)) >> 5;
    const int ix = X >> 5, iy = Y >> 5;
    const long plane = (long)img_h * img_w, pix = (long)y * img_w + x;
    float* o = out + (long)n * K * plane + pix;
    if (ix >= w || ix + 1 < 0 || iy >= h || iy + 1 < 0) {
        for (int k = 0; k < K; k++) o[k * plane] = 0.f;
        return;
    }
    const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
    const float w0 = __fmul_rn(1.f - fy, 1.f - fx), w1 = __fmul_rn(1.f - fy, fx);
    const float w2 = __fmul_rn(fy, 1.f - fx), w3 = __fmul_rn(fy, fx);
    const bool x0 = ix >= 0, x1 = ix + 1 < w, y0 = iy >= 0, y1 = iy + 1 < h;
    const float* src = hm + (long)n * K * h * w;
    for (int k = 0; k < K; k++, src += h * w) {
        const float v0 = (x0 && y0) ? src[iy * w + ix] : 0.f;
        const float v1 = (x1 && y0) ? src[iy * w + ix + 1] : 0.f;
        const float v2 = (x0 && y1) ? src[(iy + 1) * w + ix] : 0.f;
        const float v3 = (x1 && y1) ? src[(iy + 1) * w + ix + 1] : 0.f;
        float v = __fmul_rn(v0, w0);
        v = __fadd_rn(v, __fmul_rn(v1, w1));
        v = __fadd_rn(v, __fmul_rn(v2, w2));
        v = __fadd_rn(v, __fmul_rn(v3, w3));
        o[k * plane] = v;
    }
}

}  // namespace

extern "C" int mvp_preprocess(const uint8_t* frames, int n, int H, int W, const double* minv, int out_h, int out_w,
                              const float* mean3, const float* std3, int swap_rb, int with_flip, uint16_t* out,
                              void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n >= 0 && H > 0 && W > 0 && out_h > 0 && out_w > 0, "mvp_preprocess: bad sizes");
    MVP_REQUIRE(mean3 && std3, "mvp_preprocess: mean/std are NULL");
    if (n == 0) return MVP_OK;
    MVP_REQUIRE(frames && minv && out, "mvp_preprocess: NULL device pointer");
    PreParams p{};
    p.frames = frames;
    p.minv = minv;
    p.out = out;
    p.n = n;
    p.H = H;
    p.W = W;
    p.oh = out_h;
    p.ow = out_w;
    p.swap_rb = swap_rb;
    p.flip = with_flip;
    for (int c = 0; c < 3; c++) {
        p.mean[c] = mean3[c];
        p.stdv[c] = std3[c];
    }
    MVP_REQUIRE((long)out_h * out_w < (1L << 30) && n < 65536, "mvp_preprocess: sizes");
    hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)((out_h * out_w + kBlock - 1) / kBlock), (unsigned)n),
                       dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), p);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_heatmap_decode(const float* hm, const float* hm_flip, int N, int K, int H, int W,
                                  const int* flip_idx, int shift, const float* center_scale, int input_w,
                                  int input_h, float* avg_out, float* kpts, float* scores, int32_t* argmax,
                                  float* kpts_tkv, int V, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(N >= 0 && K > 0 && K <= 32 && H > 2 && W > 2, "mvp_heatmap_decode: bad sizes");
    MVP_REQUIRE(input_w > 0 && input_h > 0, "mvp_heatmap_decode: bad input size");
    if (N == 0) return MVP_OK;
    MVP_REQUIRE(hm && center_scale && kpts && scores, "mvp_heatmap_decode: NULL device pointer");
    DecodeParams p{};
    p.hm = hm;
    p.hmf = hm_flip;
    p.cs = center_scale;
    p.avg = avg_out;
    p.kpts = kpts;
    p.scores = scores;
    p.amax = argmax;
    p.tkv = kpts_tkv;
    p.V = V;
    MVP_REQUIRE(!kpts_tkv || (V > 0 && N % V == 0), "mvp_heatmap_decode: N=%d not a multiple of V=%d", N, V);
    p.N = N;
    p.K = K;
    p.H = H;
    p.W = W;
    p.shift = shift;
    p.in_w = input_w;
    p.in_h = input_h;
    for (int k = 0; k < K; k++) {
        const int f = flip_idx ? flip_idx[k] : k;
        MVP_REQUIRE(f >= 0 && f < K, "mvp_heatmap_decode: flip_idx[%d]=%d", k, f);
        p.flip_idx[k] = f;
    }
    const long maps = (long)N * K;
    hipLaunchKernelGGL(decode_kernel, dim3((unsigned)((maps + 3) / 4)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), p);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_heatmap_moments(const float* hm, int N, int K, int h, int w, const double* minv, int img_h,
                                   int img_w, float thr, int separable, const int* separable_dev, double* out,
                                   void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(N >= 0 && K > 0 && h > 0 && w > 0 && img_h > 0 && img_w > 0, "mvp_heatmap_moments: bad sizes");
    // map, 2 column tables, row table, run starts / ends, run sums (fp64): moments_kernel's layout
    const size_t lds0 = (size_t)((h * w + 3) & ~3) * 4 + (size_t)img_w * 8 + (size_t)((img_h + 2) & ~1) * 4 +
                        (size_t)((h + 2) & ~1) * 8 + (size_t)(h + 1) * 48;
    MVP_REQUIRE(lds0 <= kMomMaxLds, "mvp_heatmap_moments: map %dx%d + image %dx%d exceed the LDS budget", h, w,
                img_h, img_w);
    // the mixed-column closed forms need a 48-B prefix row per image row (separable == 1 only)
    const bool mixcf = separable == 1 && lds0 + (size_t)img_h * 48 <= kMomMaxLdsCf;
    const size_t lds = mixcf ? lds0 + (size_t)img_h * 48 : lds0;
    static bool attr = false;
    if (!attr) {
        MVP_HIP(hipFuncSetAttribute((const void*)moments_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    kMomMaxLdsCf));
        attr = true;
    }
    if (N == 0) return MVP_OK;
    MVP_REQUIRE(hm && minv && out, "mvp_heatmap_moments: NULL device pointer");
    MomParams p{};
    p.hm = hm;
    p.minv = minv;
    p.out = out;
    p.N = N;
    p.K = K;
    p.h = h;
    p.w = w;
    p.img_h = img_h;
    p.img_w = img_w;
    p.thr = thr;
    p.separable = separable;
    p.sep = separable_dev;
    p.mixcf = mixcf ? 1 : 0;
    const char* je = getenv("MVPOSE_MOM_JPB");  // tuning experiments / tests only
    const int jpb_env = je ? atoi(je) : 0;
    p.jpb = jpb_env > 0 ? std::min(jpb_env, K) : std::min(kMomJointsPerBlock, K);
    const long groups = (K + p.jpb - 1) / p.jpb;
    hipLaunchKernelGGL(moments_kernel, dim3((unsigned)((long)N * groups)), dim3(kMomBlock), lds,
                       reinterpret_cast<hipStream_t>(stream), p);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_heatmap_revert(const float* hm, int N, int K, int h, int w, const double* minv, int img_h,
                                  int img_w, float* out, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(N >= 0 && K > 0 && h > 0 && w > 0 && img_h > 0 && img_w > 0 && img_h < 65536,
                "mvp_heatmap_revert: bad sizes");
    if (N == 0) return MVP_OK;
    MVP_REQUIRE(hm && minv && out, "mvp_heatmap_revert: NULL device pointer");
    hipLaunchKernelGGL(revert_kernel, dim3((unsigned)((img_w + kBlock - 1) / kBlock), (unsigned)img_h, (unsigned)N),
                       dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), hm, minv, out, K, h, w, img_h, img_w);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}
