// Device-side person-box hand-off and top-down crop geometry.
//
// The reference's PoseEstimator.predict takes the first person box of mmdet's
// detections with score > bbox_thr, else the whole image (mmpose_pose_estimation.py:
// 242-250), and hands it to inference_topdown (:253), whose TopdownAffine derives the
// crop from it: mmpose bbox_xyxy2cs (padding 1.25) -> _fix_aspect_ratio (192:256) ->
// get_warp_matrix -> cv2.getAffineTransform (a 6x6 system solved by cv::solve's LU) ->
// cv2.warpAffine's internal inversion; revert_heatmap does the same for the 48x64
// heatmap (inv=True).  This kernel runs that chain for every camera-frame of a batch
// on the device, straight from the detector's per-frame best box, so the pipeline with
// the detector in front never synchronises with the host.  Its host twin is
// mvpose/geometry.py::crop_geometry_batch: the same fp64 / f32 operations in the same
// order with contraction off, so the two agree bit for bit (tests/test_geometry_gpu.py).
// One wave per box: every lane forms the (tiny) geometry redundantly, then the lanes
// split the separability scan of the revert map (mvp_warp_is_separable's test) that
// selects moments_kernel's column-resident path per crop.
#include "mvp_common.h"

#include <cfloat>

#pragma clang fp contract(off)

namespace {

constexpr int kInW = 192, kInH = 256;  // HRNet-W32 crop (w, h)
constexpr int kHmW = 48, kHmH = 64;    // heatmap (w, h)

// mmpose get_warp_matrix's three point pairs (rot 0, shift 0, fix_aspect_ratio), with
// the f32 rounding points of its float32 arrays (geometry._warp_points).
__device__ inline void warp_points(float cx, float cy, float sw, int out_w, int out_h, float s[3][2],
                                   float d[3][2]) {
    s[0][0] = cx;
    s[0][1] = cy;
    s[1][0] = (float)((double)cx + (double)sw * -0.5);
    s[1][1] = cy;
    const float dx = s[0][0] - s[1][0], dy = s[0][1] - s[1][1];
    s[2][0] = s[1][0] + -dy;
    s[2][1] = s[1][1] + dx;
    d[0][0] = (float)(out_w * 0.5);
    d[0][1] = (float)(out_h * 0.5);
    d[1][0] = (float)(out_w * 0.5 + out_w * -0.5);
    d[1][1] = (float)(out_h * 0.5);
    const float ex = d[0][0] - d[1][0], ey = d[0][1] - d[1][1];
    d[2][0] = d[1][0] + -ey;
    d[2][1] = d[1][1] + ex;
}

// cv2.getAffineTransform(src, dst): rows (x, y, 1, 0, 0, 0) / (0, 0, 0, x, y, 1) per point,
// solved by OpenCV's LUImpl (first row with the largest |pivot|, d = -1 / pivot, rows
// a += (a_ji d) a_i, back substitution; a pivot < 100 DBL_EPSILON = failure = zeros).
// Fully unrolled: the pivot row swap is a select per row, so the system stays in VGPRs.
__device__ inline void affine_lu(const float s[3][2], const float d[3][2], double M[6]) {
    double a[6][6], b[6];
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int c = 0; c < 6; c++) a[2 * i][c] = a[2 * i + 1][c] = 0.0;
        a[2 * i][0] = a[2 * i + 1][3] = s[i][0];
        a[2 * i][1] = a[2 * i + 1][4] = s[i][1];
        a[2 * i][2] = a[2 * i + 1][5] = 1.0;
        b[2 * i] = d[i][0];
        b[2 * i + 1] = d[i][1];
    }
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        int k = i;
        double best = fabs(a[i][i]);
#pragma unroll
        for (int j = i + 1; j < 6; j++) {
            const double v = fabs(a[j][i]);
            if (v > best) {
                best = v;
                k = j;
            }
        }
        bad |= best < 100.0 * DBL_EPSILON;
#pragma unroll
        for (int j = i + 1; j < 6; j++) {
            const bool sw = j == k;
#pragma unroll
            for (int c = 0; c < 6; c++) {
                const double t = a[i][c];
                a[i][c] = sw ? a[j][c] : t;
                a[j][c] = sw ? t : a[j][c];
            }
            const double t = b[i];
            b[i] = sw ? b[j] : t;
            b[j] = sw ? t : b[j];
        }
        const double dd = -1.0 / a[i][i];
#pragma unroll
        for (int j = i + 1; j < 6; j++) {
            const double alpha = a[j][i] * dd;
#pragma unroll
            for (int c = i + 1; c < 6; c++) a[j][c] += alpha * a[i][c];
            b[j] += alpha * b[i];
        }
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s_ = b[i];
#pragma unroll
        for (int c = i + 1; c < 6; c++) s_ -= a[i][c] * b[c];
        b[i] = s_ / a[i][i];
    }
#pragma unroll
    for (int q = 0; q < 6; q++) M[q] = bad ? 0.0 : b[q];
}

// cv2.warpAffine's inversion of M when WARP_INVERSE_MAP is not set (imgwarp.cpp, fp64).
__device__ inline void inverse_map(double m[6]) {
    double D = m[0] * m[4] - m[1] * m[3];
    D = D != 0.0 ? 1.0 / D : 0.0;
    const double a11 = m[4] * D, a22 = m[0] * D;
    m[0] = a11;
    m[4] = a22;
    m[1] *= -D;
    m[3] *= -D;
    const double b1 = -m[0] * m[2] - m[1] * m[5];
    const double b2 = -m[3] * m[2] - m[4] * m[5];
    m[2] = b1;
    m[5] = b2;
}

__global__ __launch_bounds__(64) void bbox_geometry_kernel(const float* __restrict__ boxes, int stride, int n,
                                                           int score_col, float thr, int fh, int fw,
                                                           double* __restrict__ crop_minv,
                                                           double* __restrict__ revert_minv,
                                                           float* __restrict__ center_scale, int* __restrict__ sep) {
    const int i = blockIdx.x;
    if (i >= n) return;
    const float* bx = boxes + (long)i * stride;
    float x1 = bx[0], y1 = bx[1], x2 = bx[2], y2 = bx[3];
    bool use = isfinite(x1) && isfinite(y1) && isfinite(x2) && isfinite(y2);
    if (score_col >= 0) use = use && bx[score_col] > thr;  // the hand-off rule: score > bbox_thr
    if (!use) {                                             // no person box: the whole image
        x1 = 0.f;
        y1 = 0.f;
        x2 = (float)fw;
        y2 = (float)fh;
    }
    // bbox_xyxy2cs on f32 boxes: f32 sums / differences (exact in fp64, rounded once)
    const float cx = (float)((double)x1 + (double)x2) * 0.5f;
    const float cy = (float)((double)y1 + (double)y2) * 0.5f;
    float sw = (float)((double)x2 - (double)x1) * 1.25f;
    float sh = (float)((double)y2 - (double)y1) * 1.25f;
    {  // _fix_aspect_ratio(scale, 192 / 256)
        const double w = sw, h = sh, ar = (double)kInW / (double)kInH;
        if (w > h * ar) {
            sw = (float)w;
            sh = (float)(w / ar);
        } else {
            sw = (float)(h * ar);
            sh = (float)h;
        }
    }
    float s[3][2], d[3][2];
    double cm[6], rm[6];
    warp_points(cx, cy, sw, kInW, kInH, s, d);
    affine_lu(s, d, cm);  // image -> crop
    inverse_map(cm);      // crop -> image (what warpAffine samples with)
    warp_points(cx, cy, sw, kHmW, kHmH, s, d);
    affine_lu(d, s, rm);  // heatmap -> image (revert_heatmap, inv=True)
    inverse_map(rm);      // image -> heatmap
    const int lane = threadIdx.x;
    if (lane < 6) {
        crop_minv[6 * i + lane] = cm[lane];
        revert_minv[6 * i + lane] = rm[lane];
    }
    if (lane == 0) {
        center_scale[4 * i + 0] = cx;
        center_scale[4 * i + 1] = cy;
        center_scale[4 * i + 2] = sw;
        center_scale[4 * i + 3] = sh;
    }
    // separability of the fixed-point revert warp (mvp_warp_is_separable): source column
    // independent of y, source row independent of x
    bool ok = true;
    const int X00 = (int)rint((rm[1] * 0 + rm[2]) * 1024.0);
    for (int y = 1 + lane; y < fh; y += 64) ok &= (int)rint((rm[1] * y + rm[2]) * 1024.0) == X00;
    const int b0 = (int)rint(rm[3] * 0 * 1024.0);
    for (int x = 1 + lane; x < fw; x += 64) ok &= (int)rint(rm[3] * x * 1024.0) == b0;
    const bool all_ok = !__any(!ok);
    if (lane == 0) sep[i] = all_ok ? 1 : 0;
}

}  // namespace

extern "C" int mvp_bbox_geometry(const float* boxes, int stride, int n, int score_col, float bbox_thr, int frame_h,
                                 int frame_w, double* crop_minv, double* revert_minv, float* center_scale,
                                 int* separable, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n >= 0 && stride >= 4 && score_col < stride && frame_h > 0 && frame_w > 0,
                "mvp_bbox_geometry: bad arguments (n=%d stride=%d score_col=%d frame %dx%d)", n, stride, score_col,
                frame_h, frame_w);
    if (n == 0) return MVP_OK;
    MVP_REQUIRE(boxes && crop_minv && revert_minv && center_scale && separable, "mvp_bbox_geometry: NULL pointer");
    hipLaunchKernelGGL(bbox_geometry_kernel, dim3((unsigned)n), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       boxes, stride, n, score_col, bbox_thr, frame_h, frame_w, crop_minv, revert_minv, center_scale,
                       separable);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}
