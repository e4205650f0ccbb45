// Batched multi-view triangulation for gfx950 — one (frame, joint) problem per lane.
//
// Replaces the reference's T*J Python-level calls of utils.triangulate_points
// (pose_estimation.py:27-53 -> utils.py:1277-1336), whose numerics live in
// OpenCV 4.9 (cv.undistortPoints, cv.triangulatePoints,
// cv.convertPointsFromHomogeneous).  Per lane, in fp64 with no FMA contraction
// so the rounding sequence is OpenCV's:
//   1. undistort each view's (x, y) with its own K/dist: 5 fixed iterations,
//      icdist<0 fallback, RR = K, rounded to f32 (cvUndistortPointsInternal);
//   2. A (2V x 4): rows x·P[2]-P[0], y·P[2]-P[1] per view (icvTriangulatePoints);
//   3. null vector = Vt row 3 of cv::SVD (JacobiSVDImpl_): by default computed by
//      Householder QR + inverse iteration to the fp64 noise floor (qr_inverse_iteration,
//      ~1/4 of the FP64 work), falling back per lane to the exact restatement —
//      one-sided Hestenes Jacobi on the rows of Aᵀ, eps = 10·DBL_EPSILON,
//      descending selection sort — when that iteration has not provably
//      converged; MVP_TRI_EXACT_JACOBI forces the restatement for every lane;
//   4. f32 homogeneous divide: s = w != 0 ? 1.f/w : 1.f (convertPointsFromHomogeneous).
// The reference's camera selection (top-2 by confidence, ascending; parameters
// keyed by selection position; pose_estimation.py:32-45) is reproduced in
// MVP_TRI_REFERENCE mode.
//
// Roofline: HBM-bound by design at 12·(V+1) B per point (read x,y,conf per view,
// write xyz) but FP64-issue-heavy (Jacobi ≈ 2-3 kFLOP/point); see DESIGN.md.
#pragma clang fp contract(off)

#include "mvp_common.h"

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

namespace {

constexpr int kMaxCams = 8;
constexpr int kBlock = 256;

struct CamIdx {
    int v[kMaxCams];
};

// cvUndistortPointsInternal (OpenCV 4.9), R = I, P = K, 5 iterations, 5 coefficients.
// The k4..k6 / thin-prism terms are zero and contribute exact zeros; they are
// omitted (sign-of-zero differences cannot change the result).  OpenCV computes in
// double and stores into the source's depth: undistort_point rounds to f32 (CV_32FC2
// keypoints, the pipeline), undistort_point_f64 keeps the double (CV_64FC2).
__device__ __forceinline__ void undistort_point_f64(double u, double v, const double* __restrict__ c,
                                                    double& ox, double& oy) {
    const double fx = c[0], fy = c[4];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double cx = c[2], cy = c[5];
    const double k0 = c[9], k1 = c[10], k2 = c[11], k3 = c[12], k4 = c[13];
    double x = (u - cx) * ifx;
    double y = (v - cy) * ify;
    const double x0 = x, y0 = y;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = 1. / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        if (icdist < 0) {
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x);
        double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    double xx = c[0] * x + c[1] * y + c[2];
    double yy = c[3] * x + c[4] * y + c[5];
    double ww = 1. / (c[6] * x + c[7] * y + c[8]);
    ox = xx * ww;
    oy = yy * ww;
}

__device__ __forceinline__ void undistort_point(float uf, float vf, const double* __restrict__ c,
                                                float& ox, float& oy) {
    double x, y;
    undistort_point_f64(uf, vf, c, x, y);
    ox = (float)x;
    oy = (float)y;
}

// 1/b with the arithmetic of the compiler's IEEE fp64 division (v_div_scale,
// v_rcp_f64, two Newton steps, one quotient correction, v_div_fmas, v_div_fixup)
// minus the scale / fixup instructions, which are identities for finite, normal
// b away from the exponent limits: bit-identical there, 7 instructions not 11.
// Used for every reciprocal of the fast path; every b here is O(1) to O(1e6).
__device__ __forceinline__ double recip_rn(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(e, r, r);
}

// sqrt(s) for s > 0 by v_rsq_f64 + two Goldschmidt steps + one residual
// correction (~1 ulp); the fast solver's norms only.
__device__ __forceinline__ double sqrt_fast(double s) {
    const double y = __builtin_amdgcn_rsq(s);
    double g = s * y, h = 0.5 * y;
    double r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double d = __builtin_fma(-g, g, s);
    return s > 0 ? __builtin_fma(d, h, g) : 0.0;
}

// 1/sqrt(s), s > 0, to ~1 ulp: v_rsq_f64 + two Newton steps.
__device__ __forceinline__ double rsqrt_fast(double s) {
    double y = __builtin_amdgcn_rsq(s);
    double t = s * y;
    double e = __builtin_fma(-t, y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    t = s * y;
    e = __builtin_fma(-t, y, 1.0);
    return __builtin_fma(0.5 * y, e, y);
}

// Per-camera constants of the fast undistortion, computed once per block with
// the same IEEE operations the per-point code would do (1./fx, 1./fy).
struct CamFast {
    double ifx, ify;
};

// undistort_point with the loop-invariant reciprocals from CamFast and every
// division as recip_rn; branch-free, so the two views of a point interleave.
// Same operation sequence and rounding as undistort_point for finite input.
__device__ __forceinline__ void undistort_point_fast(float uf, float vf, const double* __restrict__ c,
                                                     const CamFast& cf, float& ox, float& oy) {
    const double cx = c[2], cy = c[5];
    const double k0 = c[9], k1 = c[10], k2 = c[11], k3 = c[12], k4 = c[13];
    const double u = uf, v = vf;
    double x = (u - cx) * cf.ifx;
    double y = (v - cy) * cf.ify;
    const double x0 = x, y0 = y;
    bool neg = false;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = recip_rn(1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        neg = neg || (icdist < 0);
        double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x);
        double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // OpenCV breaks out with the initial guess on icdist < 0: the iterates after
    // such a step are discarded here instead — selects, not a branch, so both
    // views' chains stay in one basic block for the scheduler to interleave
    // (the branch form measured 0.081 vs 0.058 ms per 1.7 M points)
    x = neg ? x0 : x;
    y = neg ? y0 : y;
    double xx = c[0] * x + c[1] * y + c[2];
    double yy = c[3] * x + c[4] * y + c[5];
    const double ww = recip_rn(c[6] * x + c[7] * y + c[8]);
    ox = (float)(xx * ww);
    oy = (float)(yy * ww);
}

// std::hypot as OpenCV's JacobiSVDImpl_ gets it from libm on Linux: glibc 2.35's __ieee754_hypot
// (sysdeps/ieee754/dbl-64/e_hypot.c, the non-FMA kernel x86-64 builds; verified bit-identical to
// this image's libm on 5e7 random pairs, tests/test_oracle_triangulate.py).  The compiler's
// hypot (ocml) rounds differently in the last bit, which made ~60 % of the exact path's float64
// outputs differ from the restatement's in round 4.
__device__ __forceinline__ double hypot_kernel(double ax, double ay) {
    double h = sqrt(ax * ax + ay * ay);
    double t1, t2;
    if (h <= 2.0 * ay) {
        const double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        const double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

__device__ __noinline__ double hypot_glibc(double x, double y) {
    if (!isfinite(x) || !isfinite(y)) {
        if (isinf(x) || isinf(y)) return INFINITY;
        return x + y;
    }
    x = fabs(x);
    y = fabs(y);
    const double ax = x < y ? y : x, ay = x < y ? x : y;
    if (ax > 0x1p+511) {
        if (ay <= ax * 0x1p-54) return ax + ay;
        return hypot_kernel(ax * 0x1p-600, ay * 0x1p-600) / 0x1p-600;
    }
    if (ay < 0x1p-511) {
        if (ax >= ay / 0x1p-54) return ax + ay;
        return hypot_kernel(ax / 0x1p-600, ay / 0x1p-600) * 0x1p-600;
    }
    if (ay <= ax * 0x1p-54) return ax + ay;
    return hypot_kernel(ax, ay);
}

// JacobiSVDImpl_<double> on At (4 rows of length M); returns Vt row of the
// smallest singular value after OpenCV's descending selection sort.
template <int M>
__device__ __forceinline__ void jacobi_null_vector(double (&At)[4][M], double (&nv)[4]) {
    double W[4];
    double Vt[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < 4; k++) Vt[i][k] = (i == k) ? 1.0 : 0.0;
    }
    const double eps = DBL_EPSILON * 10;
    const int max_iter = M > 30 ? M : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 3; i++) {
#pragma unroll
            for (int j = i + 1; j < 4; j++) {
                double a = W[i], b = W[j], p = 0;
#pragma unroll
                for (int k = 0; k < M; k++) p += At[i][k] * At[j][k];
                if (!(fabs(p) <= eps * sqrt(a * b))) {
                    p *= 2;
                    double beta = a - b, gamma = hypot_glibc(p, beta);
                    double c, s;
                    if (beta < 0) {
                        double delta = (gamma - beta) * 0.5;
                        s = sqrt(delta / gamma);
                        c = p / (gamma * s * 2);
                    } else {
                        c = sqrt((gamma + beta) / (gamma * 2));
                        s = p / (gamma * c * 2);
                    }
                    a = 0;
                    b = 0;
#pragma unroll
                    for (int k = 0; k < M; k++) {
                        double t0 = c * At[i][k] + s * At[j][k];
                        double t1 = -s * At[i][k] + c * At[j][k];
                        At[i][k] = t0;
                        At[j][k] = t1;
                        a += t0 * t0;
                        b += t1 * t1;
                    }
                    W[i] = a;
                    W[j] = b;
                    changed = true;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        double t0 = c * Vt[i][k] + s * Vt[j][k];
                        double t1 = -s * Vt[i][k] + c * Vt[j][k];
                        Vt[i][k] = t0;
                        Vt[j][k] = t1;
                    }
                }
            }
        }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
    // descending selection sort (only the Vt rows matter), compile-time row indices
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < 4; k++)
            if (wj < W[k]) {
                wj = W[k];
                j = k;
            }
#pragma unroll
        for (int k = i + 1; k < 4; k++)
            if (j == k) {
                double t = W[i];
                W[i] = W[k];
                W[k] = t;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    double tv = Vt[i][q];
                    Vt[i][q] = Vt[k][q];
                    Vt[k][q] = tv;
                }
            }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) nv[q] = Vt[3][q];
}

// Certification of the throughput solvers against the exact path (OpenCV's rounding sequence).
// A float64 value c that the exact path rounds to float32 (cvmSet into the f32 points4D, the f32
// undistorted points) is computed here with an error |e| <= delta.  If c lies farther than
// 2·delta from the f32 rounding midpoint nearest it, float(c + e) == float(c): both paths store
// the same bits.  That midpoint has c's sign, exponent and upper 23 mantissa bits and mantissa bit
// 28 set (one v_and_or_b32); c - m is exact (Sterbenz).  The factor 2 covers the finer f32 grid
// just below a power of two.  NaN / Inf / 0 / f32-subnormal c never pass (|c - m| is NaN or
// below any delta used here).
__device__ __forceinline__ bool f32_rounding_stable(double c, double delta2) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(c);
    const unsigned long long mb = (b & 0xFFFFFFFFE0000000ull) | 0x10000000ull;
    return fabs(c - __longlong_as_double((long long)mb)) > delta2;
}

// Error bound of a certified null vector (unit vector, absolute per component):
//   8 · (remaining inverse-iteration error, estimated as step² / previous step: the iterate's
//        off-null component shrinks by the same factor λ₄/λ₃ each step; sqrt(dd) once the
//        steps stop contracting, i.e. at the rounding floor)
// + 0.2 · eps · sqrt(tr M / D₂) (rounding floor of both solvers; eps·σ₁/σ₃ with D₂ the third
//        LDLᵀ pivot of M = AᵀA standing in for λ₃: the exact Jacobi's own error measured
//        <= 0.025 of it, the normal equations' floor <= 0.0033, D₂/λ₃ <= 1.4, on 1.4 M synthetic
//        and random points: tools/tri_cert_emu.c — an EMPIRICAL bound, not a proof; the GPU
//        tests add adversarial rigs: tiny baselines, points near the epipoles)
// + 2^-50 (normalisation).  Returned doubled for f32_rounding_stable.
__device__ __forceinline__ double null_vector_delta2(double dd, double prev, double cond2) {
    const float d = (float)dd, pv = (float)prev;
    const float it_err = d * __builtin_amdgcn_rsqf(fmaxf(fmaxf(d, pv), 1e-37f));
    return (double)(16.f * it_err + 0.4f * 2.220446e-16f * __builtin_sqrtf((float)cond2) + 0x1p-49f);
}

__device__ __forceinline__ bool null_vector_certified(const double (&nv)[4], double delta2) {
    return f32_rounding_stable(nv[0], delta2) && f32_rounding_stable(nv[1], delta2) &&
           f32_rounding_stable(nv[2], delta2) && f32_rounding_stable(nv[3], delta2);
}

// Fast null vector of A (M x 4): Householder QR (A = QR; R is 4x4 upper
// triangular with A's right singular vectors), then inverse iteration on RᵀR
// started from R⁻¹e₄.  Each step shrinks the component off the smallest right
// singular vector by (σ₄/σ₃)² (~1e-6 on real rigs), so two or three steps reach
// the fp64 noise floor, where the unit vector agrees with JacobiSVDImpl_'s Vt
// row 3 to ~1e-13 (its own rounding error) at a fraction of the FP64 work.
// Returns false unless the iteration has provably converged (ill-conditioned
// geometry with σ₄ ≈ σ₃, NaN/Inf input) AND its f32-rounded components are certified equal
// to the Jacobi restatement's (null_vector_certified): the caller then runs the exact Jacobi
// restatement, so the default solver's outputs are bit-identical to the exact path's.  FMA contraction is allowed here: this is an approximation of the
// Jacobi result, checked by its own convergence test, not a restatement of
// OpenCV's rounding sequence.
template <int M>
__device__ __forceinline__ bool qr_inverse_iteration(const double (&A0)[M][4], double (&nv)[4]) {
#pragma clang fp contract(fast)
    double A[M][4];
#pragma unroll
    for (int r = 0; r < M; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) A[r][c] = A0[r][c];
    double R[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        double s = 0;
#pragma unroll
        for (int r = k; r < M; r++) s += A[r][k] * A[r][k];
        const double nrm = sqrt_fast(s);
        if (k == 3) {
            R[3][3] = nrm;
            break;
        }
        const double akk = A[k][k];
        const double alpha = akk >= 0 ? -nrm : nrm;
        // reflector v = a - alpha·e_k; vᵀv / 2 = nrm (nrm + |akk|)
        const double half_vtv = nrm * (nrm + fabs(akk));
        const double inv = half_vtv > 0 ? recip_rn(half_vtv) : 0.0;
        A[k][k] = akk - alpha;
        R[k][k] = alpha;
#pragma unroll
        for (int j = k + 1; j < 4; j++) {
            double d = 0;
#pragma unroll
            for (int r = k; r < M; r++) d += A[r][k] * A[r][j];
            const double t = d * inv;
#pragma unroll
            for (int r = k; r < M; r++) A[r][j] -= t * A[r][k];
            R[k][j] = A[k][j];
        }
    }
    // an exactly singular R (noise-free data): a perturbation far below the QR
    // rounding error keeps R⁻¹ finite and changes nothing else
    const double scale = fmax(fmax(fabs(R[0][0]), fabs(R[1][1])), fabs(R[2][2]));
    if (fabs(R[3][3]) < 1e-18 * scale) R[3][3] = 1e-18 * scale;
    double d[4];
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = recip_rn(R[k][k]);
    auto back = [&](double (&x)[4]) {  // x <- R⁻¹ x
        x[3] = x[3] * d[3];
        x[2] = (x[2] - R[2][3] * x[3]) * d[2];
        x[1] = (x[1] - R[1][2] * x[2] - R[1][3] * x[3]) * d[1];
        x[0] = (x[0] - R[0][1] * x[1] - R[0][2] * x[2] - R[0][3] * x[3]) * d[0];
    };
    auto fwd = [&](double (&x)[4]) {  // x <- R⁻ᵀ x
        x[0] = x[0] * d[0];
        x[1] = (x[1] - R[0][1] * x[0]) * d[1];
        x[2] = (x[2] - R[0][2] * x[0] - R[1][2] * x[1]) * d[2];
        x[3] = (x[3] - R[0][3] * x[0] - R[1][3] * x[1] - R[2][3] * x[2]) * d[3];
    };
    auto normalize = [&](double (&x)[4]) {
        const double is = rsqrt_fast(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] *= is;
    };
    double x[4] = {0.0, 0.0, 0.0, 1.0};
    back(x);
    normalize(x);
    double prev = 1.0;  // squared step length of the previous iteration
    for (int it = 0; it < 12; it++) {
        double y[4] = {x[0], x[1], x[2], x[3]};
        fwd(y);
        back(y);
        normalize(y);  // (RᵀR)⁻¹ is positive definite: no sign flip between iterates
        double dd = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double e = y[q] - x[q];
            dd += e * e;
            x[q] = y[q];
        }
        // squared step dd; geometric convergence: remaining error ≈ step · (step / prev),
        // i.e. step <= 4e-16, or step <= 1e-6 and step² <= 1e-14 · prev
        if (dd <= 1.6e-31 || (dd <= 1e-12 && dd * dd <= 1e-28 * prev)) {
#pragma unroll
            for (int q = 0; q < 4; q++) nv[q] = x[q];
            // certified against the exact path, else its Jacobi: RᵀR = AᵀA, so tr M = ‖R‖²_F
            // and the third LDLᵀ pivot is R₂₂²
            double trm = 0;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = i; j < 4; j++) trm += R[i][j] * R[i][j];
            return null_vector_certified(nv, null_vector_delta2(dd, prev, trm * d[2] * d[2]));
        }
        if (it >= 2 && !(dd < 0.25 * prev)) return false;  // not contracting (or NaN)
        prev = dd;
    }
    return false;
}

__device__ __forceinline__ void write_result(const double (&nv)[4], int64_t p, float* __restrict__ out,
                                             double* __restrict__ out4) {
    // cvmSet into the f32 points4D, then convertPointsFromHomogeneous in f32.
    const float X = (float)nv[0], Y = (float)nv[1], Z = (float)nv[2], w = (float)nv[3];
    const float s = (w != 0.f) ? __frcp_rn(w) : 1.f;
    out[3 * p + 0] = __fmul_rn(X, s);
    out[3 * p + 1] = __fmul_rn(Y, s);
    out[3 * p + 2] = __fmul_rn(Z, s);
    if (out4) {
        out4[4 * p + 0] = nv[0];
        out4[4 * p + 1] = nv[1];
        out4[4 * p + 2] = nv[2];
        out4[4 * p + 3] = nv[3];
    }
}

__device__ __forceinline__ void add_view_rows(double (*A)[4], int r, double x, double y,
                                              const double* __restrict__ P) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        A[r][k] = x * P[8 + k] - P[0 + k];
        A[r + 1][k] = y * P[8 + k] - P[4 + k];
    }
}

__device__ __forceinline__ void load_cams(double (*scam)[MVP_CAM_DOUBLES], CamFast* sfast,
                                          const double* __restrict__ cams, int n_cams) {
    const int total = n_cams * MVP_CAM_DOUBLES;
    for (int i = threadIdx.x; i < total; i += blockDim.x) scam[i / MVP_CAM_DOUBLES][i % MVP_CAM_DOUBLES] = cams[i];
    if (threadIdx.x < n_cams) {
        const double* c = cams + threadIdx.x * MVP_CAM_DOUBLES;
        sfast[threadIdx.x].ifx = 1. / c[0];
        sfast[threadIdx.x].ify = 1. / c[4];
    }
    __syncthreads();
}

// ----------------------------------------------------------------- tolerance mode
// MVP_TRI_TOLERANCE: the reference-mode two-camera problem solved for throughput, with every
// output CERTIFIED bit-identical to the exact path (OpenCV's rounding sequence); a point that
// cannot be certified is re-solved on the exact path by a second launch.
//   * undistortion: OpenCV's 5 fixed iterations.  The first NF32 run in f32 (both views packed
//     in v_pk_* instructions) on the distortion correction c = x - x0 rather than on x, so the
//     f32 rounding error scales with |c| ~ |k1| r² |x| instead of |x|; the rest run in fp64 from
//     x0 + c.  Bound: the f32 iterates' error <= kappa · 2^-24 · (the terms' magnitudes), carried
//     through each fp64 iteration by L, a bound on the iteration map's Jacobian at the last f32
//     iterate (the distortion polynomial's derivative and the tangential terms), plus the fp64
//     rounding; the f64 undistorted pixel is certified when it lies farther than that bound from
//     an f32 rounding midpoint (f32_rounding_stable): its f32 rounding is then the exact path's;
//   * null vector: normal equations M = AᵀA (fp64), LDLᵀ, inverse iteration from M⁻¹e₄ to a
//     geometric convergence test (2-5 steps; each shrinks the off-null component by
//     λ₄/λ₃ = (σ₄/σ₃)², median 4e-7 on the synthetic rigs); certified by null_vector_delta2;
//   * the camera at the world origin (P = [K | 0], the reference's camera 0,
//     setup_camera_configuration.py:392-393) contributes 6 non-zero entries to M, 3 of them per-
//     camera constants: M is formed from its two rows in closed form (21 fewer fp64 operations);
//   * not certified, not contracting (σ₄ ≈ σ₃ geometry), Inf input, a distortion denominator
//     near zero (OpenCV's icdist < 0 branch): the exact path (fallback launch).  NaN input is
//     answered inline (the exact path gives NaN for every output).
// The certified result is dehomogenised through OpenCV's f32 chain (write_result, shared).
// Measured rates (tests/test_triangulate_gpu.py prints them): see DESIGN.md §4.2.

typedef float f2v __attribute__((ext_vector_type(2)));

struct CamTol {              // per-camera constants of the f32 iterations and the error bound
    float k1, k2, k3;        // radial
    float p1, p2, p1x2, p2x2;  // tangential, and doubled
    float a1, a2, a3, b;     // Jacobian bound: 2|k1|, 4|k2|, 6|k3|, 8(|p1| + |p2|)
    float kn;                // |fx| + |skew| + |fy|: pixels per normalised unit
    float floor2;            // 2 · 2^-45 (|cx| + |cy|): the K application's rounding near cx, cy
    int ok;                  // K's last row is (0, 0, 1) and fx, fy != 0: the pixel bound holds
    int origin;              // P = [K | 0] with K's last row (0, 0, 1) and K[1][0] == 0
};

__device__ __forceinline__ CamTol make_cam_tol(const double* __restrict__ c) {
    CamTol t;
    const double k1 = c[9], k2 = c[10], p1 = c[11], p2 = c[12], k3 = c[13];
    t.k1 = (float)k1;
    t.k2 = (float)k2;
    t.k3 = (float)k3;
    t.p1 = (float)p1;
    t.p2 = (float)p2;
    t.p1x2 = (float)(2 * p1);
    t.p2x2 = (float)(2 * p2);
    t.a1 = (float)(2 * fabs(k1)) * 1.0001f;
    t.a2 = (float)(4 * fabs(k2)) * 1.0001f;
    t.a3 = (float)(6 * fabs(k3)) * 1.0001f;
    t.b = (float)(8 * (fabs(p1) + fabs(p2))) * 1.0001f;
    t.kn = (float)(fabs(c[0]) + fabs(c[1]) + fabs(c[4])) * 1.0001f;
    t.floor2 = (float)(0x1p-44 * (fabs(c[2]) + fabs(c[5])));
    t.ok = c[6] == 0 && c[7] == 0 && c[8] == 1 && c[0] != 0 && c[4] != 0;
    const double* P = c + 26;
    t.origin = t.ok && c[3] == 0 && P[3] == 0 && P[7] == 0 && P[11] == 0 && P[8] == 0 && P[9] == 0 && P[10] == 1 &&
               P[4] == 0 && P[0] == c[0] && P[1] == c[1] && P[2] == c[2] && P[5] == c[4] && P[6] == c[5];
    return t;
}

// r = 1/b to ~1 ulp: v_rcp_f64 + two Newton steps (no IEEE-division scaling)
__device__ __forceinline__ double rcp_nr(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(r, e, r);
}

// r = 1/b to ~11 ulp: v_rcp_f64 (~2^-24) + one Newton step (profiles/r03p_rcp_probe.log).
// For the undistortion's fp64 steps: 11 ulp of fp64 is ~1e-15 relative, inside the bound's
// fp64 term.
__device__ __forceinline__ double rcp_nr1(double b) {
    const double r = __builtin_amdgcn_rcp(b);
    return __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
}

// Both views of a point: (u, v) pixels -> undistorted pixels (P = K), OpenCV's iteration, the
// first NF32 of the 5 in f32 on the correction, the rest in fp64.  ox / oy: the f32 values;
// certified &= both views' values provably equal the exact path's.
template <int NF32>
__device__ __forceinline__ void undistort_pair_tol(const float (&u)[2], const float (&v)[2],
                                                   const double* __restrict__ c0, const double* __restrict__ c1,
                                                   const CamFast& f0, const CamFast& f1, const CamTol& t0,
                                                   const CamTol& t1, float (&ox)[2], float (&oy)[2],
                                                   bool& certified) {
#pragma clang fp contract(fast)
    constexpr int NF64 = 5 - NF32;
    const double* cc[2] = {c0, c1};
    double x0[2], y0[2];
    x0[0] = ((double)u[0] - c0[2]) * f0.ifx;
    y0[0] = ((double)v[0] - c0[5]) * f0.ify;
    x0[1] = ((double)u[1] - c1[2]) * f1.ifx;
    y0[1] = ((double)v[1] - c1[5]) * f1.ify;
    const f2v X0 = {(float)x0[0], (float)x0[1]}, Y0 = {(float)y0[0], (float)y0[1]};
    const f2v K1 = {t0.k1, t1.k1}, K2 = {t0.k2, t1.k2}, K3 = {t0.k3, t1.k3};
    const f2v P1 = {t0.p1, t1.p1}, P2 = {t0.p2, t1.p2}, P1x2 = {t0.p1x2, t1.p1x2}, P2x2 = {t0.p2x2, t1.p2x2};
    const f2v one = {1.f, 1.f}, two = {2.f, 2.f};
    f2v cx = {0.f, 0.f}, cy = {0.f, 0.f}, x = X0, y = Y0, r2 = {0.f, 0.f}, poly = {0.f, 0.f};
    f2v ic = {1.f, 1.f}, dX = {0.f, 0.f}, dY = {0.f, 0.f};
    f2v den_min = {1.f, 1.f};
#pragma unroll
    for (int j = 0; j < NF32; j++) {
        x = X0 + cx;
        y = Y0 + cy;
        r2 = __builtin_elementwise_fma(x, x, y * y);
        poly = r2 * __builtin_elementwise_fma(__builtin_elementwise_fma(K3, r2, K2), r2, K1);
        const f2v den = poly + one;
        den_min = __builtin_elementwise_min(den_min, den);
        ic.x = __builtin_amdgcn_rcpf(den.x);
        ic.y = __builtin_amdgcn_rcpf(den.y);
        const f2v xy = x * y;
        dX = __builtin_elementwise_fma(P1x2, xy, P2 * __builtin_elementwise_fma(two * x, x, r2));
        dY = __builtin_elementwise_fma(P1, __builtin_elementwise_fma(two * y, y, r2), P2x2 * xy);
        cx = -(__builtin_elementwise_fma(X0, poly, dX) * ic);
        cy = -(__builtin_elementwise_fma(Y0, poly, dY) * ic);
    }
    // error of the f32 correction: kappa = 8 roundings of the terms it is built from (X0 and the
    // iterate x rounded to f32, poly, the tangential terms, the approximate reciprocal),
    // propagated through each later iteration by L.  Scalar f32 (|.| is a free source modifier
    // there; packed instructions would need an and-mask per absolute value).  |x| + |y| <=
    // 0.5 + r² bounds the tangential Jacobian's (|x| + |y|) factor without absolute values.
    const CamTol* tt[2] = {&t0, &t1};
    float errq[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const float r2q = q ? r2.y : r2.x, icq = q ? ic.y : ic.x, pq = q ? poly.y : poly.x;
        const float L = icq * __builtin_fmaf(r2q, __builtin_fmaf(__builtin_fmaf(tt[q]->a3, r2q, tt[q]->a2), r2q, tt[q]->a1),
                                             tt[q]->b * (0.5f + r2q));
        const float terms = __builtin_fmaf(fabsf(q ? X0.y : X0.x) + fabsf(q ? Y0.y : Y0.x), fabsf(pq),
                                           fabsf(q ? dX.y : dX.x) + fabsf(q ? dY.y : dY.x));
        float e = (8.f * 0x1p-24f) * terms * icq;
#pragma unroll
        for (int j = 0; j < NF64; j++) e *= L;
        errq[q] = e;
    }
    double xd[2] = {x0[0] + (double)cx.x, x0[1] + (double)cx.y};
    double yd[2] = {y0[0] + (double)cy.x, y0[1] + (double)cy.y};
    double dmin[2] = {(double)den_min.x, (double)den_min.y};
#pragma unroll
    for (int j = NF32; j < 5; j++) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const double* c = cc[q];
            const double k1 = c[9], k2 = c[10], p1 = c[11], p2 = c[12], k3 = c[13];
            const double rr = xd[q] * xd[q] + yd[q] * yd[q];
            const double den = 1 + ((k3 * rr + k2) * rr + k1) * rr;
            dmin[q] = fmin(dmin[q], den);
            const double icd = rcp_nr1(den);
            const double ddX = 2 * p1 * xd[q] * yd[q] + p2 * (rr + 2 * xd[q] * xd[q]);
            const double ddY = p1 * (rr + 2 * yd[q] * yd[q]) + 2 * p2 * xd[q] * yd[q];
            xd[q] = (x0[q] - ddX) * icd;
            yd[q] = (y0[q] - ddY) * icd;
        }
    }
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const double* c = cc[q];
        const double ww = rcp_nr1(c[6] * xd[q] + c[7] * yd[q] + c[8]);
        const double oxd = (c[0] * xd[q] + c[1] * yd[q] + c[2]) * ww;
        const double oyd = (c[3] * xd[q] + c[4] * yd[q] + c[5]) * ww;
        ox[q] = (float)oxd;
        oy[q] = (float)oyd;
        // pixel error bound, doubled: kn · (the f32 error carried through) + 2^-44 (|ox| + |oy|)
        // + floor2 (2^-44 (|cx| + |cy|)): the fp64 iterations' and the K application's rounding
        // (kn |x| <= |ox| + |cx|, so this covers 2^-46 kn |x| with a factor 4)
        const double d2 = __builtin_fma(0x1p-44, fabs(oxd) + fabs(oyd), (double)(2.f * tt[q]->kn * errq[q] + tt[q]->floor2));
        // OpenCV's icdist < 0 branch (keep the initial guess) and a near-zero denominator are left
        // to the exact path: the f32 and fp64 denominators could disagree on the sign
        certified = certified && tt[q]->ok && dmin[q] > 0x1p-10 && f32_rounding_stable(oxd, d2) &&
                    f32_rounding_stable(oyd, d2);
    }
}

// Null vector of M = AᵀA (lower triangle m[i][j], j <= i) by LDLᵀ inverse iteration; false = not
// provably converged or not certified against the exact path.
__device__ __forceinline__ bool normal_eq_null_vector(const double (&m)[4][4], double (&nv)[4]) {
#pragma clang fp contract(fast)
    // LDLᵀ (lower triangle of m)
    const double D0 = m[0][0], r0 = rcp_nr(D0);
    const double l10 = m[1][0] * r0, l20 = m[2][0] * r0, l30 = m[3][0] * r0;
    const double a11 = m[1][1] - l10 * m[1][0], a21 = m[2][1] - l20 * m[1][0], a31 = m[3][1] - l30 * m[1][0];
    const double a22 = m[2][2] - l20 * m[2][0], a32 = m[3][2] - l30 * m[2][0], a33 = m[3][3] - l30 * m[3][0];
    const double r1 = rcp_nr(a11);
    const double l21 = a21 * r1, l31 = a31 * r1;
    const double b22 = a22 - l21 * a21, b32 = a32 - l31 * a21, b33 = a33 - l31 * a31;
    const double r2 = rcp_nr(b22);
    const double l32 = b32 * r2;
    double D3 = b33 - l32 * b32;
    // an exactly singular M (noise-free data): the last pivot is rounding noise of either sign;
    // a positive pivot far below the factorisation's rounding keeps the solves finite and M⁻¹
    // positive definite (a negative one flipped the iterate's sign every step, so 27 % of the
    // noise-free points never converged) and changes nothing else
    if (!(D3 >= 1e-30 * D0)) D3 = 1e-30 * D0;
    const double r3 = rcp_nr(D3);
    auto solve = [&](double (&y)[4]) {  // y <- M⁻¹ y
        const double z1 = y[1] - l10 * y[0];
        const double z2 = y[2] - l20 * y[0] - l21 * z1;
        const double z3 = y[3] - l30 * y[0] - l31 * z1 - l32 * z2;
        y[3] = z3 * r3;
        y[2] = z2 * r2 - l32 * y[3];
        y[1] = z1 * r1 - l21 * y[2] - l31 * y[3];
        y[0] = y[0] * r0 - l10 * y[1] - l20 * y[2] - l30 * y[3];
    };
    double x[4];
    x[3] = r3;  // M⁻¹ e₄
    x[2] = -l32 * x[3];
    x[1] = -l21 * x[2] - l31 * x[3];
    x[0] = -l10 * x[1] - l20 * x[2] - l30 * x[3];
    {
        const double is = rsqrt_fast(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] *= is;
    }
    // e₄ is a poor start (the null vector is (X, Y, Z, 1)/|.| with |X, Y, Z| ~ 1e2-1e3 world
    // units, so its e₄ component is ~1/350) and λ₄/λ₃ reaches ~2e-5 on the synthetic rigs:
    // iterate to a geometric convergence test (remaining error ≈ step · step / previous step
    // <= 1e-13).  Branch-free per lane: every lane takes the same steps (a converged lane stays
    // converged), two unconditionally, more only while some lane of the wave is still
    // contracting — the per-lane early exits compiled to ~40 register copies per step.
    auto step = [&](double& dd) {
        double y[4] = {x[0], x[1], x[2], x[3]};
        solve(y);
        const double is = rsqrt_fast(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
        dd = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            y[q] *= is;  // M⁻¹ is positive definite (up to the pivot clamp): no sign flip
            const double e = y[q] - x[q];
            dd += e * e;
            x[q] = y[q];
        }
    };
    auto converged = [](double dd, double prev) { return dd <= 1e-26 || (dd <= 1e-16 && dd * dd <= 1e-26 * prev); };
    double d0, d1;
    step(d0);
    step(d1);
    bool ok = converged(d1, d0) || converged(d0, 1.0);
    bool failed = false;
    double prev = d0, last = d1;
#pragma unroll 1
    for (int it = 2; it < 8 && __builtin_amdgcn_ballot_w64(!ok && !failed) != 0; it++) {
        double dd;
        step(dd);
        const bool now = converged(dd, last);
        failed = failed || (!ok && !now && !(dd < 0.25 * last));  // not contracting (or NaN)
        ok = ok || now;
        prev = last;
        last = dd;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) nv[q] = x[q];
    // certification: the rounding floor uses tr M / D₂ (D₂ = b22, the third pivot)
    const double cond2 = (m[0][0] + m[1][1] + (m[2][2] + m[3][3])) * r2;
    return ok && !failed && null_vector_certified(nv, null_vector_delta2(last, prev, cond2));
}

// Solver stages.  kExact: the restatement for every lane (OpenCV undistortion
// with IEEE divisions, Jacobi SVD).  kFast: fast undistortion (the same rounding) + QR /
// inverse iteration, with the Jacobi restatement (on the same A) for the lanes whose
// iteration has not provably converged or whose f32 outputs are not certified equal to the
// restatement's (null_vector_certified): bit-identical to kExact.
//
// Measured and dropped (tools/pmc_tri.sh, V=2, 1.7 M points): moving the Jacobi
// fallback to a second launch over marked lanes cuts the fast kernel from 110 to
// 66 VGPRs (4 -> 7 waves per SIMD) but made it slower (69 vs 58 us; VALU busy
// 59 % vs 73 %), and the marker sweep cost another 23 us.
enum Stage { kExact = 0, kFast = 1, kTol = 2 };

template <int S>
__device__ __forceinline__ void undistort_view(float u, float v, const double* __restrict__ c, const CamFast& cf,
                                               float& ox, float& oy) {
    if constexpr (S == kExact)
        undistort_point(u, v, c, ox, oy);
    else
        undistort_point_fast(u, v, c, cf, ox, oy);
}

template <int S, int M>
__device__ __forceinline__ void solve_and_write(const double (&A)[M][4], int64_t p, float* __restrict__ out,
                                                double* __restrict__ out4) {
    double nv[4];
    if (S == kExact || !qr_inverse_iteration<M>(A, nv)) {
        double At[4][M];
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int r = 0; r < M; r++) At[c][r] = A[r][c];
        jacobi_null_vector<M>(At, nv);
    }
    write_result(nv, p, out, out4);
}

// MVP_TRI_REFERENCE: top-2 listed cameras by confidence (ascending), params keyed
// by selection position (reference quirk, pose_estimation.py:36-45).
template <int S>
__device__ __forceinline__ void triangulate_reference_body(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams,
    CamIdx ci, int n_ci, float* __restrict__ out, double* __restrict__ out4) {
    __shared__ double scam[kMaxCams][MVP_CAM_DOUBLES];
    __shared__ CamFast sfast[kMaxCams];
    load_cams(scam, sfast, cams, n_cams);
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const float* __restrict__ kp = kpts + p * 3 * V;
    // stable ascending argsort, NaN last; keep the last two (pose_estimation.py:36)
    int best = 0, second = -1;
    float cbest = kp[2 * V + ci.v[0]];
    float csecond = 0.f;
#pragma unroll
    for (int i = 1; i < kMaxCams; i++) {
        if (i < n_ci) {
            const float c = kp[2 * V + ci.v[i]];
            const bool after_best = isnan(c) ? true : (isnan(cbest) ? false : (c >= cbest));
            if (after_best) {
                second = best;
                csecond = cbest;
                best = i;
                cbest = c;
            } else {
                const bool after_second =
                    (second < 0) ? true : (isnan(c) ? true : (isnan(csecond) ? false : (c >= csecond)));
                if (after_second) {
                    second = i;
                    csecond = c;
                }
            }
        }
    }
    const int pos0 = second, pos1 = best;  // top_indices = [lower-conf, higher-conf]
    const int col0 = ci.v[pos0], col1 = ci.v[pos1];
    float u0x, u0y, u1x, u1y;
    // points come from the selected columns; parameters from camera key = position
    undistort_view<S>(kp[col0], kp[V + col0], scam[pos0], sfast[pos0], u0x, u0y);
    undistort_view<S>(kp[col1], kp[V + col1], scam[pos1], sfast[pos1], u1x, u1y);
    double A[4][4];
    add_view_rows(A, 0, u0x, u0y, scam[pos0] + 26);
    add_view_rows(A, 2, u1x, u1y, scam[pos1] + 26);
    solve_and_write<S, 4>(A, p, out, out4);
}

// MVP_TRI_ALL_VIEWS: one 2·NV x 4 DLT over the NV listed views.
template <int S, int NV>
__device__ __forceinline__ void triangulate_all_views_body(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams,
    CamIdx ci, float* __restrict__ out, double* __restrict__ out4) {
    __shared__ double scam[kMaxCams][MVP_CAM_DOUBLES];
    __shared__ CamFast sfast[kMaxCams];
    load_cams(scam, sfast, cams, n_cams);
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const float* __restrict__ kp = kpts + p * 3 * V;
    double A[2 * NV][4];
#pragma unroll
    for (int j = 0; j < NV; j++) {
        const int col = ci.v[j];
        float ux, uy;
        undistort_view<S>(kp[col], kp[V + col], scam[col], sfast[col], ux, uy);
        add_view_rows(A, 2 * j, ux, uy, scam[col] + 26);
    }
    solve_and_write<S, 2 * NV>(A, p, out, out4);
}

template <int S>
__global__ __launch_bounds__(kBlock) void triangulate_reference_kernel(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams, CamIdx ci,
    int n_ci, float* __restrict__ out, double* __restrict__ out4) {
    triangulate_reference_body<S>(kpts, n, V, cams, n_cams, ci, n_ci, out, out4);
}

template <int S, int NV>
__global__ __launch_bounds__(kBlock) void triangulate_all_views_kernel(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams, CamIdx ci,
    float* __restrict__ out, double* __restrict__ out4) {
    triangulate_all_views_body<S, NV>(kpts, n, V, cams, n_cams, ci, out, out4);
}

// MVP_TRI_REFERENCE | MVP_TRI_TOLERANCE with camera_indices of length 2 (the reference's
// hard-coded [0, 1]): the top-2 rule reduces to one comparison (np.argsort of two values:
// [0, 1] unless conf[1] < conf[0], NaN sorts last).
struct Tol2Sel {
    int pos0, pos1;
    float u[2], v[2];
};
__device__ __forceinline__ Tol2Sel tol2_select(const float* __restrict__ kp, int V, const CamIdx& ci) {
    const int ca = ci.v[0], cb = ci.v[1];
    const float conf_a = kp[2 * V + ca], conf_b = kp[2 * V + cb];
    // stable ascending argsort of (conf_a, conf_b), NaN last: swapped iff conf_b sorts before conf_a
    const bool swap = isnan(conf_a) ? !isnan(conf_b) : (conf_b < conf_a);
    // rows of the lower-confidence camera first; each view's point comes from its column
    // ci.v[pos] and its parameters from camera key = its position pos in camera_indices
    Tol2Sel r;
    r.pos0 = swap ? 1 : 0;
    r.pos1 = swap ? 0 : 1;
    const int col0 = ci.v[r.pos0], col1 = ci.v[r.pos1];
    r.u[0] = kp[col0];
    r.u[1] = kp[col1];
    r.v[0] = kp[V + col0];
    r.v[1] = kp[V + col1];
    return r;
}

// Points the tolerance kernel could not certify are re-solved on the exact path by a second
// launch, so the exact path's registers (Jacobi on A^T and V^T: the inline fallback held the
// kernel at 150 VGPRs = 3 waves per SIMD) never limit the occupancy of the throughput kernel.
// The tolerance kernel marks such a point's x output with a signalling-NaN sentinel (arithmetic
// never produces it) and appends its index to a per-stream list (one atomic per wave); past the
// list's capacity the fallback sweeps the outputs for the sentinel instead.  The fallback grid
// (kFbBlocks workgroups, one exact point per lane at a time) adds its count to a running total
// (mvp_triangulate_fallback_total) and its last workgroup resets the list for the next launch.
constexpr int kFbCap = 1 << 16;
constexpr int kFbBlocks = 128;
constexpr uint32_t kFbSentinel = 0x7FA5A5A5u;

struct FbHeader {
    unsigned count;            // entries appended by the current launch
    unsigned done;             // fallback workgroups finished (the last one resets)
    unsigned long long total;  // points re-solved on this stream since the list was created
};

struct FbList {
    FbHeader* hdr;
    unsigned* idx;  // [kFbCap]
    int force;      // tests: send every finite point to the fallback (MVPOSE_TRI_FORCE_FALLBACK=1)
};

// M = AᵀA (lower triangle) of the two views' DLT rows x·P₂ - P₀, y·P₂ - P₁ (FMA-contracted:
// any rounding is inside the certification's floor).  ORIGIN = 1: view 0's camera has P = [K | 0]
// with K's last row (0, 0, 1): its rows are (-fx, -s, du, 0) and (0, -fy, dv, 0) with du = x - cx,
// dv = y - cy (the values the generic rows hold) and its part of M is fx², fx·s, s² + fy²
// (constants), -fx·du, -(s·du + fy·dv), du² + dv².
template <bool ORIGIN>
__device__ __forceinline__ void normal_matrix_2v(const double (&x)[2], const double (&y)[2],
                                                 const double* __restrict__ c0, const double* __restrict__ c1,
                                                 double (&m)[4][4]) {
#pragma clang fp contract(fast)
    double a[2][4], b[2][4];
#pragma unroll
    for (int q = ORIGIN ? 1 : 0; q < 2; q++) {
        const double* P = (q == 0 ? c0 : c1) + 26;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            a[q][k] = __builtin_fma(x[q], P[8 + k], -P[0 + k]);
            b[q][k] = __builtin_fma(y[q], P[8 + k], -P[4 + k]);
        }
    }
    if constexpr (ORIGIN) {
        const double fx = c0[0], s = c0[1], fy = c0[4];
        const double du = x[0] - c0[2], dv = y[0] - c0[5];
        double m0[4][4] = {};
        m0[0][0] = fx * fx;
        m0[1][0] = fx * s;
        m0[1][1] = s * s + fy * fy;
        m0[2][0] = -fx * du;
        m0[2][1] = -(s * du + fy * dv);
        m0[2][2] = du * du + dv * dv;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j <= i; j++)
                m[i][j] = __builtin_fma(a[1][i], a[1][j], __builtin_fma(b[1][i], b[1][j], m0[i][j]));
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) {
                double t = a[0][i] * a[0][j];
                t = __builtin_fma(b[0][i], b[0][j], t);
                t = __builtin_fma(a[1][i], a[1][j], t);
                m[i][j] = __builtin_fma(b[1][i], b[1][j], t);
            }
    }
}

// Grid-stride: a grid of (CUs x resident blocks per CU) blocks loops over the points, so the
// per-block set-up (camera records into LDS, their reciprocals and bound constants) is paid once
// per resident block instead of once per 256 points.  The point's live state is ~100 VGPRs; 5
// waves per SIMD (96 VGPRs, 4 spilled) measured 0.500 ms per 1 M frames against 0.525 for one
// point per thread at 5 waves and 0.556 at 4 (same box, gpurun_out/r05b).
template <int NF32>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void triangulate_tol2_kernel(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams, CamIdx ci,
    float* __restrict__ out, double* __restrict__ out4, FbList fb) {
    __shared__ double scam[kMaxCams][MVP_CAM_DOUBLES];
    __shared__ CamFast sfast[kMaxCams];
    __shared__ CamTol stol[2];
    load_cams(scam, sfast, cams, n_cams);
    if (threadIdx.x < 2) stol[threadIdx.x] = make_cam_tol(cams + threadIdx.x * MVP_CAM_DOUBLES);
    __syncthreads();
    // the camera at the world origin (block-uniform): its rows in closed form, whichever order
    // the confidences put the two views in (the order only changes M's rounding)
    const int origin = stol[0].origin ? 0 : (stol[1].origin ? 1 : -1);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += stride) {
        const Tol2Sel sel = tol2_select(kpts + p * 3 * V, V, ci);
        const double* cp[2] = {scam[sel.pos0], scam[sel.pos1]};
        bool ok;
        if (isnan(sel.u[0]) || isnan(sel.u[1]) || isnan(sel.v[0]) || isnan(sel.v[1])) {
            // a NaN coordinate makes every entry of its view's rows, hence the whole SVD, NaN on
            // the exact path: all outputs NaN
            const double qn = __builtin_nan("");
            const double nv[4] = {qn, qn, qn, qn};
            write_result(nv, p, out, out4);
            ok = true;
        } else {
            float ux[2], uy[2];
            bool cert = !fb.force;
            undistort_pair_tol<NF32>(sel.u, sel.v, cp[0], cp[1], sfast[sel.pos0], sfast[sel.pos1], stol[sel.pos0],
                                     stol[sel.pos1], ux, uy, cert);
            double m[4][4];
            if (origin >= 0) {
                const int io = sel.pos0 == origin ? 0 : 1;  // the origin camera's view slot
                const double xs[2] = {(double)(io == 0 ? ux[0] : ux[1]), (double)(io == 0 ? ux[1] : ux[0])};
                const double ys[2] = {(double)(io == 0 ? uy[0] : uy[1]), (double)(io == 0 ? uy[1] : uy[0])};
                normal_matrix_2v<true>(xs, ys, scam[origin], scam[1 - origin], m);
            } else {
                const double xs[2] = {(double)ux[0], (double)ux[1]}, ys[2] = {(double)uy[0], (double)uy[1]};
                normal_matrix_2v<false>(xs, ys, cp[0], cp[1], m);
            }
            double nv[4];
            ok = normal_eq_null_vector(m, nv) && cert;
            if (ok) write_result(nv, p, out, out4);
            else reinterpret_cast<unsigned*>(out)[3 * p] = kFbSentinel;
        }
        // wave-aggregated append of the uncertified points
        const unsigned long long msk = __ballot(!ok);
        if (msk) {
            const int lane = __lane_id();
            const int leader = __ffsll((long long)msk) - 1;
            unsigned base = 0;
            if (lane == leader) base = atomicAdd(&fb.hdr->count, (unsigned)__popcll(msk));
            base = __shfl(base, leader);
            if (!ok) {
                const unsigned slot = base + (unsigned)__popcll(msk & ((1ull << lane) - 1));
                if (slot < (unsigned)kFbCap) fb.idx[slot] = (unsigned)p;
            }
        }
    }
}

// The exact path (OpenCV undistortion with IEEE divisions, Jacobi SVD) for one point.
__device__ __forceinline__ void tol2_exact_point(const float* __restrict__ kpts, int64_t p, int V,
                                              const double (*scam)[MVP_CAM_DOUBLES], const CamIdx& ci,
                                              float* __restrict__ out, double* __restrict__ out4) {
    const Tol2Sel sel = tol2_select(kpts + p * 3 * V, V, ci);
    const double* cp[2] = {scam[sel.pos0], scam[sel.pos1]};
    float e0x, e0y, e1x, e1y;
    undistort_point(sel.u[0], sel.v[0], cp[0], e0x, e0y);
    undistort_point(sel.u[1], sel.v[1], cp[1], e1x, e1y);
    double E[4][4];
    add_view_rows(E, 0, e0x, e0y, cp[0] + 26);
    add_view_rows(E, 2, e1x, e1y, cp[1] + 26);
    double At[4][4];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int r = 0; r < 4; r++) At[c][r] = E[r][c];
    double nv[4];
    jacobi_null_vector<4>(At, nv);
    write_result(nv, p, out, out4);
}

// kFbBlocks workgroups: the listed points (or, past the list's capacity, every point whose x
// output carries the sentinel), strided over the grid; the last workgroup to finish adds the
// count to the running total and resets the list for the next launch on the stream.  Every
// workgroup reads the count before it signals `done`, so the reset cannot race a reader.
__global__ __launch_bounds__(kBlock) void triangulate_tol2_fallback_kernel(
    const float* __restrict__ kpts, int64_t n, int V, const double* __restrict__ cams, int n_cams, CamIdx ci,
    float* __restrict__ out, double* __restrict__ out4, FbList fb) {
    __shared__ double scam[kMaxCams][MVP_CAM_DOUBLES];
    __shared__ CamFast sfast[kMaxCams];
    const unsigned cnt = __atomic_load_n(&fb.hdr->count, __ATOMIC_RELAXED);
    if (cnt == 0) return;  // the usual case: nothing to re-solve, the count is already 0
    load_cams(scam, sfast, cams, n_cams);
    const unsigned stride = gridDim.x * kBlock;
    if (cnt <= (unsigned)kFbCap) {
        for (unsigned i = blockIdx.x * kBlock + threadIdx.x; i < cnt; i += stride) {
            const unsigned p = fb.idx[i];
            if ((int64_t)p < n) tol2_exact_point(kpts, p, V, scam, ci, out, out4);  // never write past this call's n
        }
    } else {
        const unsigned* ob = reinterpret_cast<const unsigned*>(out);
        for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += stride)
            if (ob[3 * p] == kFbSentinel) tol2_exact_point(kpts, p, V, scam, ci, out, out4);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&fb.hdr->done, 1u) == gridDim.x - 1) {
            fb.hdr->total += cnt;
            fb.hdr->count = 0u;
            fb.hdr->done = 0u;
            __threadfence();
        }
    }
}

// utils.triangulate_points (utils.py:1277-1336) on float64 keypoints, as the extrinsic
// branch calls it on its Gaussian samples (pose_refinement.py:811): cv.undistortPoints keeps
// CV_64F (no f32 rounding of the undistorted points), cv.triangulatePoints builds the same
// fp64 A and writes a CV_64F points4D, cv.convertPointsFromHomogeneous divides in double
// (scale = w != 0 ? 1./w : 1.).  kpts: (n, 2 views, 2) [point][view][x, y]; cams: the two
// views' records (camera 1 first).  Exact Jacobi restatement for every point.
__global__ __launch_bounds__(kBlock) void triangulate_pairs_f64_kernel(const double* __restrict__ kpts, int64_t n,
                                                                       const double* __restrict__ cams,
                                                                       double* __restrict__ out,
                                                                       double* __restrict__ out4) {
    __shared__ double scam[2][MVP_CAM_DOUBLES];
    for (int i = threadIdx.x; i < 2 * MVP_CAM_DOUBLES; i += blockDim.x) scam[i / MVP_CAM_DOUBLES][i % MVP_CAM_DOUBLES] = cams[i];
    __syncthreads();
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const double* k = kpts + 4 * p;
    double E[4][4];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        double ex, ey;
        undistort_point_f64(k[2 * q], k[2 * q + 1], scam[q], ex, ey);
        add_view_rows(E, 2 * q, ex, ey, scam[q] + 26);
    }
    double At[4][4];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int r = 0; r < 4; r++) At[c][r] = E[r][c];
    double nv[4];
    jacobi_null_vector<4>(At, nv);
    const double w = nv[3];
    const double s = (w != 0.) ? 1. / w : 1.;
    out[3 * p + 0] = nv[0] * s;
    out[3 * p + 1] = nv[1] * s;
    out[3 * p + 2] = nv[2] * s;
    if (out4) {
#pragma unroll
        for (int q = 0; q < 4; q++) out4[4 * p + q] = nv[q];
    }
}

// The tolerance kernel's fallback list, one per (device, stream), allocated on first use
// (a stream-captured launch needs one uncaptured call on that stream first).  The list is
// shared by every call on its stream, so a call holds the list's own mutex from the first
// launch to the second: two host threads on one stream (PyTorch's default stream is shared)
// then enqueue tol A, fallback A, tol B, fallback B, never tol A, tol B, fallback A, ...
struct FbSlot {
    FbList fb;
    std::mutex* mu;
};

FbSlot tol_fallback_list(hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, FbSlot> lists;
    int dev = 0;
    MVP_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(mu);
    auto it = lists.find({dev, s});
    if (it != lists.end()) return it->second;
    void* buf = nullptr;
    MVP_HIP(hipMalloc(&buf, sizeof(FbHeader) + (size_t)kFbCap * sizeof(unsigned)));
    MVP_HIP(hipMemsetAsync(buf, 0, sizeof(FbHeader), s));
    FbHeader* hdr = static_cast<FbHeader*>(buf);
    const FbSlot slot{FbList{hdr, reinterpret_cast<unsigned*>(hdr + 1), 0}, new std::mutex};  // lives as long as the process
    lists[{dev, s}] = slot;
    return slot;
}

}  // namespace

extern "C" int mvp_triangulate(const float* kpts, int64_t n_points, int V, const double* cams, int n_cams,
                               const int* cam_idx, int n_cam_idx, int mode, float* out_xyz, double* out_xyzw,
                               void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n_points >= 0, "mvp_triangulate: n_points < 0");
    MVP_REQUIRE(V >= 2 && V <= 64, "mvp_triangulate: V=%d out of range", V);
    MVP_REQUIRE(n_cams >= 1 && n_cams <= kMaxCams, "mvp_triangulate: n_cams=%d (1..%d)", n_cams, kMaxCams);
    MVP_REQUIRE(cam_idx != nullptr, "mvp_triangulate: cam_idx is NULL");
    MVP_REQUIRE(n_cam_idx >= 2 && n_cam_idx <= kMaxCams, "mvp_triangulate: n_cam_idx=%d (2..%d)", n_cam_idx,
                kMaxCams);
    CamIdx ci{};
    for (int i = 0; i < n_cam_idx; i++) {
        MVP_REQUIRE(cam_idx[i] >= 0 && cam_idx[i] < V && cam_idx[i] < n_cams,
                    "mvp_triangulate: cam_idx[%d]=%d out of range (V=%d, n_cams=%d)", i, cam_idx[i], V, n_cams);
        ci.v[i] = cam_idx[i];
    }
    if (n_points == 0) return MVP_OK;
    MVP_REQUIRE(kpts && cams && out_xyz, "mvp_triangulate: null device pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t blocks = (n_points + kBlock - 1) / kBlock;
    MVP_REQUIRE(blocks < (1LL << 31), "mvp_triangulate: too many points");
    const bool exact = (mode & MVP_TRI_EXACT_JACOBI) != 0;
    const bool tol = (mode & MVP_TRI_TOLERANCE) != 0;
    MVP_REQUIRE(!(exact && tol), "mvp_triangulate: MVP_TRI_EXACT_JACOBI and MVP_TRI_TOLERANCE exclude each other");
    mode &= ~(MVP_TRI_EXACT_JACOBI | MVP_TRI_TOLERANCE);
    const dim3 grid((unsigned)blocks), block(kBlock);
    if (mode == MVP_TRI_REFERENCE) {
        MVP_REQUIRE(n_cam_idx <= n_cams, "mvp_triangulate: reference mode keys params by position: need "
                    "n_cam_idx <= n_cams");
        if (tol && n_cam_idx == 2 && n_points < (1LL << 32)) {
            const FbSlot slot = tol_fallback_list(s);
            std::lock_guard<std::mutex> call_lock(*slot.mu);
            FbList fb = slot.fb;
            const char* ff = getenv("MVPOSE_TRI_FORCE_FALLBACK");  // tests: exercise the fallback list / sweep
            // the float64 null vectors (out_xyzw, a diagnostic output) are the exact path's only
            // when it solves every point; the certification covers the f32 outputs
            fb.force = (ff && ff[0] == '1') || out_xyzw != nullptr;
            // 3 f32 + 2 fp64 undistortion iterations: 4 + 1 sends ~0.6 % of the synthetic rigs'
            // points to the exact path (0.013 % with 3 + 2, tools/tri_cert_emu.c)
            static int cus = 0;
            if (cus == 0) {
                int dev = 0;
                MVP_HIP(hipGetDevice(&dev));
                MVP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            }
            // 5 blocks of 4 waves per CU = the kernel's 5 waves per SIMD (88 VGPRs)
            const dim3 tgrid((unsigned)std::min<int64_t>(blocks, (int64_t)cus * 5));
            hipLaunchKernelGGL(triangulate_tol2_kernel<3>, tgrid, block, 0, s, kpts, n_points, V, cams, n_cams, ci,
                               out_xyz, out_xyzw, fb);
            hipLaunchKernelGGL(triangulate_tol2_fallback_kernel, dim3(kFbBlocks), block, 0, s, kpts, n_points, V, cams,
                               n_cams, ci, out_xyz, out_xyzw, fb);
        } else if (exact)
            hipLaunchKernelGGL(triangulate_reference_kernel<kExact>, grid, block, 0, s, kpts, n_points, V, cams,
                               n_cams, ci, n_cam_idx, out_xyz, out_xyzw);
        else
            hipLaunchKernelGGL(triangulate_reference_kernel<kFast>, grid, block, 0, s, kpts, n_points, V, cams,
                               n_cams, ci, n_cam_idx, out_xyz, out_xyzw);
    } else if (mode == MVP_TRI_ALL_VIEWS) {
#define MVP_TRI_CASE(NV)                                                                                      \
    case NV:                                                                                                  \
        if (exact)                                                                                            \
            hipLaunchKernelGGL((triangulate_all_views_kernel<kExact, NV>), grid, block, 0, s, kpts, n_points, V, \
                               cams, n_cams, ci, out_xyz, out_xyzw);                                          \
        else                                                                                                  \
            hipLaunchKernelGGL((triangulate_all_views_kernel<kFast, NV>), grid, block, 0, s, kpts, n_points, V,  \
                               cams, n_cams, ci, out_xyz, out_xyzw);                                          \
        break;
        switch (n_cam_idx) {
            MVP_TRI_CASE(2)
            MVP_TRI_CASE(3)
            MVP_TRI_CASE(4)
            MVP_TRI_CASE(5)
            MVP_TRI_CASE(6)
            MVP_TRI_CASE(7)
            MVP_TRI_CASE(8)
        }
#undef MVP_TRI_CASE
    } else {
        mvp::fail(MVP_ERR_ARG, "mvp_triangulate: unknown mode %d", mode);
    }
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_triangulate_points_f64(const double* kpts_2d, int64_t n_points, const double* cams,
                                          double* out_xyz, double* out_xyzw, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n_points >= 0, "mvp_triangulate_points_f64: n_points < 0");
    if (n_points == 0) return MVP_OK;
    MVP_REQUIRE(kpts_2d && cams && out_xyz, "mvp_triangulate_points_f64: null device pointer");
    const int64_t blocks = (n_points + kBlock - 1) / kBlock;
    MVP_REQUIRE(blocks < (1LL << 31), "mvp_triangulate_points_f64: too many points");
    hipLaunchKernelGGL(triangulate_pairs_f64_kernel, dim3((unsigned)blocks), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), kpts_2d, n_points, cams, out_xyz, out_xyzw);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_triangulate_fallback_total(void* stream, unsigned long long* out_total) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(out_total != nullptr, "mvp_triangulate_fallback_total: out_total is NULL");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const FbSlot slot = tol_fallback_list(s);
    std::lock_guard<std::mutex> call_lock(*slot.mu);
    MVP_HIP(hipStreamSynchronize(s));
    MVP_HIP(hipMemcpy(out_total, &slot.fb.hdr->total, sizeof(unsigned long long), hipMemcpyDeviceToHost));
    MVP_ABI_END
}
