// Outlier-filtered local linear smoothing of a 3D trajectory — one (t, point, dim)
// sample per lane.
//
// Replaces the reference's triple Python loop linear_interpolation
// (pose_refinement.py:15-84), which the refinement CLI always runs
// (:1170-1172).  Per sample, over the window [t - k/2, t + k/2] clipped to the
// sequence, in float32 with numpy's op order (sequential small-n sums, median =
// middle of the sorted window or the f32 mean of the two middles):
//   keep  |w - mean| <= k_std·std  [&& |w - median| <= median_std·MAD]
//   < 2 kept        -> 0 (the reference `continue`s past its assignment)
//   rolling average -> f32 mean of the kept samples
//   otherwise       -> least-squares line through (time, kept) evaluated at t,
//                      float64 (np.polyfit + np.polyval), rounded to f32.
// Reads of neighbouring t are coalesced: lanes run along (point, dim), the
// contiguous axis of the [T][P][D] layout.
#pragma clang fp contract(off)

#include "mvp_common.h"

#include <cmath>

namespace {

constexpr int kMaxWin = 31;

struct InterpArgs {
    const float* pts;
    float* out;
    int T, PD, k;
    float k_std, median_std;
    int rolling, use_median;
};

__device__ __forceinline__ void sort_small(float* v, int n) {
    for (int i = 1; i < n; i++) {
        const float x = v[i];
        int j = i - 1;
        while (j >= 0 && v[j] > x) {
            v[j + 1] = v[j];
            j--;
        }
        v[j + 1] = x;
    }
}

__device__ __forceinline__ float median_small(float* v, int n) {
    sort_small(v, n);
    if (n & 1) return v[n / 2];
    return (v[n / 2 - 1] + v[n / 2]) / 2.f;
}

__global__ __launch_bounds__(256) void interp_kernel(InterpArgs a) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)a.T * a.PD) return;
    const int t = (int)(i / a.PD), e = (int)(i - (long)t * a.PD);
    const int start = max(0, t - a.k / 2), end = min(a.T, t + a.k / 2 + 1);
    const int n = end - start;
    float w[kMaxWin], s[kMaxWin];
    float sum = 0.f;
    for (int r = 0; r < n; r++) {
        w[r] = a.pts[(long)(start + r) * a.PD + e];
        sum = sum + w[r];
    }
    const float mean = sum / (float)n;
    float ss = 0.f;
    for (int r = 0; r < n; r++) {
        const float d = w[r] - mean;
        ss = ss + d * d;
    }
    const float std_ = sqrtf(ss / (float)n);
    for (int r = 0; r < n; r++) s[r] = w[r];
    const float med = median_small(s, n);
    for (int r = 0; r < n; r++) s[r] = fabsf(w[r] - med);
    const float mad = median_small(s, n);
    const float lim_mean = a.k_std * std_, lim_med = a.median_std * mad;
    int cnt = 0;
    float vsum = 0.f;
    double st = 0.0, sy = 0.0;
    unsigned keep = 0;
    for (int r = 0; r < n; r++) {
        bool ok = fabsf(w[r] - mean) <= lim_mean;
        if (a.use_median) ok = ok && (fabsf(w[r] - med) <= lim_med);
        if (!ok) continue;
        keep |= 1u << r;
        cnt++;
        vsum = vsum + w[r];
        st += (double)(start + r);
        sy += (double)w[r];
    }
    float res = 0.f;
    if (cnt >= 2) {
        if (a.rolling) {
            res = vsum / (float)cnt;
        } else {
            const double tm = st / cnt, ym = sy / cnt;
            double sxy = 0.0, sxx = 0.0;
            for (int r = 0; r < n; r++) {
                if (!(keep >> r & 1u)) continue;
                const double dt = (double)(start + r) - tm;
                sxy += dt * ((double)w[r] - ym);
                sxx += dt * dt;
            }
            const double slope = sxy / sxx;
            res = (float)(slope * (double)t + (ym - slope * tm));
        }
    }
    a.out[i] = res;
}

}  // namespace

extern "C" int mvp_linear_interpolation(const float* pts, int T, int P, int D, int k, float k_std, float median_std,
                                        int use_rolling_average, int filter_distance_from_median, float* out,
                                        void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(T >= 0 && P > 0 && D > 0, "mvp_linear_interpolation: bad shape T=%d P=%d D=%d", T, P, D);
    MVP_REQUIRE(k >= 1 && (k / 2) * 2 + 1 <= kMaxWin, "mvp_linear_interpolation: window k=%d outside [1, %d]", k,
                kMaxWin - 1);
    if (T == 0) return MVP_OK;
    MVP_REQUIRE(pts && out, "mvp_linear_interpolation: null pointer");
    InterpArgs a{pts, out, T, P * D, k, k_std, median_std, use_rolling_average, filter_distance_from_median};
    const long total = (long)T * P * D;
    hipLaunchKernelGGL(interp_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}
