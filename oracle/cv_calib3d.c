/*
 * ORACLE — test infrastructure only. Never linked into, loaded by, or called
 * from the product path (libmvpose.so / mvpose).  Only tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg may use it.
 *
 * CPU restatement (plain C, fp64 inside, f32 at the same rounding points) of
 * the three OpenCV 4.9.0 calib3d calls the reference's triangulation leaf
 * makes (reference utils.py:1314-1331, called once per (frame, joint) from
 * pose_estimation.py:52):
 *
 *   cv.undistortPoints(pts, K, dist, None, K)   utils.py:1314-1315
 *   cv.triangulatePoints(P1, P2, x1, x2)        utils.py:1326
 *   cv.convertPointsFromHomogeneous(X4)         utils.py:1331
 *
 * OpenCV (opencv_python==4.9.0.80, reference requirements.txt:5) is an
 * external dependency absent from /root/reference and from this image, so the
 * algorithms below restate its published source:
 *   - undistort.dispatch.cpp cvUndistortPointsInternal with
 *     TermCriteria(MAX_ITER, 5, 0.01), R = identity, P = K (RR = K·I = K);
 *   - triangulate.cpp icvTriangulatePoints: fp64 4x4 A, rows
 *     (x·P[2]-P[0], y·P[2]-P[1]) per view, cv::SVD::compute, X = Vt row 3,
 *     stored into the f32 output Mat (cvmSet casts to float);
 *   - lapack.cpp JacobiSVDImpl_<double> (one-sided Hestenes Jacobi on the
 *     rows of Aᵀ, eps = 10·DBL_EPSILON, max_iter = max(m, 30), descending
 *     sort of singular values);
 *   - fundam.cpp convertPointsFromHomogeneous (f32: scale = w != 0 ? 1.f/w : 1).
 * Parity against real cv2 is UNPINNED in this container (no cv2); it is
 * cross-checked against the reference's own utils.DLT (utils.py:19-34) at zero
 * distortion and against the reference's forward model project_points_torch
 * (pose_refinement.py:94-179) with distortion (tests/test_oracle_triangulate.py).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA contraction, so the
 * rounding sequence is the one the C source spells).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <float.h>

/* ---- cv::undistortPoints (OpenCV 4.9, R=None, P=K) ---------------------- */
/* k[0..13] = (k1,k2,p1,p2,k3,k4,k5,k6,s1,s2,s3,s4,tx,ty); tilt (tx,ty) unsupported (must be 0). */
static void undistort_one(double u, double v, const double A[3][3], const double k[14],
                          int n_iter, double* ox, double* oy)
{
    const double fx = A[0][0], fy = A[1][1];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double cx = A[0][2], cy = A[1][2];
    double x = u, y = v, x0, y0;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    /* invMatTilt = I: vecUntilt = (x, y, 1), invProj = 1 -> x0 = x, y0 = y (exact) */
    x0 = x; y0 = y;
    for (int j = 0; j < n_iter; j++) {
        double r2 = x * x + y * y;
        double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                        (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {  /* OpenCV regression_14583 fallback */
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    /* RR = P(3x3) * I = K exactly */
    double xx = A[0][0] * x + A[0][1] * y + A[0][2];
    double yy = A[1][0] * x + A[1][1] * y + A[1][2];
    double ww = 1. / (A[2][0] * x + A[2][1] * y + A[2][2]);
    *ox = xx * ww;
    *oy = yy * ww;
}

/* src, dst: n x 2 interleaved f32 (CV_32FC2). K: 9 doubles row-major. dist: ndist doubles. */
void orc_undistort_points_f32(const float* src, int64_t n, const double* K, const double* dist,
                              int ndist, float* dst)
{
    double A[3][3], k[14];
    memset(k, 0, sizeof(k));
    for (int i = 0; i < 9; i++) A[i / 3][i % 3] = K[i];
    for (int i = 0; i < ndist && i < 14; i++) k[i] = dist[i];
    for (int64_t i = 0; i < n; i++) {
        double ox, oy;
        undistort_one((double)src[2 * i], (double)src[2 * i + 1], A, k, 5, &ox, &oy);
        dst[2 * i] = (float)ox;
        dst[2 * i + 1] = (float)oy;
    }
}

/* CV_64FC2 keypoints: cvUndistortPointsInternal stores the doubles unrounded
 * (the extrinsic branch's Gaussian samples, pose_refinement.py:811). */
void orc_undistort_points_f64(const double* src, int64_t n, const double* K, const double* dist,
                              int ndist, double* dst)
{
    double A[3][3], k[14];
    memset(k, 0, sizeof(k));
    for (int i = 0; i < 9; i++) A[i / 3][i % 3] = K[i];
    for (int i = 0; i < ndist && i < 14; i++) k[i] = dist[i];
    for (int64_t i = 0; i < n; i++)
        undistort_one(src[2 * i], src[2 * i + 1], A, k, 5, &dst[2 * i], &dst[2 * i + 1]);
}

/* ---- glibc 2.35 __ieee754_hypot restated (sysdeps/ieee754/dbl-64/e_hypot.c, non-FMA kernel) ---
 * The oracle's Jacobi calls libm's hypot, as OpenCV's does; this restatement is the text the
 * device's exact path (csrc/triangulate.hip hypot_glibc) follows, checked against libm by
 * tests/test_oracle_triangulate.py. */
static double orc_hypot_kernel(double ax, double ay)
{
    double h = sqrt(ax * ax + ay * ay), t1, t2;
    if (h <= 2.0 * ay) {
        double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

double orc_hypot_restated(double x, double y)
{
    if (!isfinite(x) || !isfinite(y)) {
        if (isinf(x) || isinf(y)) return INFINITY;
        return x + y;
    }
    x = fabs(x);
    y = fabs(y);
    double ax = x < y ? y : x, ay = x < y ? x : y;
    if (ax > 0x1p+511) {
        if (ay <= ax * 0x1p-54) return ax + ay;
        return orc_hypot_kernel(ax * 0x1p-600, ay * 0x1p-600) / 0x1p-600;
    }
    if (ay < 0x1p-511) {
        if (ax >= ay / 0x1p-54) return ax + ay;
        return orc_hypot_kernel(ax / 0x1p-600, ay / 0x1p-600) * 0x1p-600;
    }
    if (ay <= ax * 0x1p-54) return ax + ay;
    return orc_hypot_kernel(ax, ay);
}

/* n pairs -> number of pairs where the restatement differs from libm's hypot */
int64_t orc_hypot_check(const double* x, const double* y, int64_t n)
{
    int64_t bad = 0;
    for (int64_t i = 0; i < n; i++) {
        double a = hypot(x[i], y[i]), b = orc_hypot_restated(x[i], y[i]);
        if (memcmp(&a, &b, sizeof a) != 0) bad++;
    }
    return bad;
}

/* ---- lapack.cpp JacobiSVDImpl_<double>, Vt only ------------------------- */
/* At: n rows of length m (row stride m), i.e. At = Aᵀ for A (m x n).  Vt: n x n. */
void orc_jacobi_svd(double* At, int m, int n, double* Wout, double* Vt)
{
    double W[16];
    const double eps = DBL_EPSILON * 10;
    int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0; Aj[k] = t1;
                    a += t0 * t0; b += t1 * t1;
                }
                W[i] = a; W[j] = b;
                changed = 1;
                double *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (int k = 0; k < n; k++) {
                    double t0 = c * Vi[k] + s * Vj[k];
                    double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0; Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < m; k++) { t = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = t; }
            for (int k = 0; k < n; k++) { t = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = t; }
        }
    }
    if (Wout) for (int i = 0; i < n; i++) Wout[i] = W[i];
}

/* ---- triangulate.cpp icvTriangulatePoints generalised to nv views ------ */
/* Ps: nv x 12 doubles (3x4 row-major).  xs: nv x n x 2 f32 (per view, per point).
 * out4: 4 x n f32 (cv's points4D layout).  nv == 2 is exactly cv::triangulatePoints. */
void orc_triangulate_nview(const double* Ps, int nv, const float* xs, int64_t n, float* out4,
                           double* out4_f64)
{
    double At[4 * 32], Vt[16];
    const int m = 2 * nv;
    for (int64_t i = 0; i < n; i++) {
        double A[32][4];
        for (int j = 0; j < nv; j++) {
            const double* P = Ps + 12 * j;
            double x = (double)xs[(j * n + i) * 2 + 0];
            double y = (double)xs[(j * n + i) * 2 + 1];
            for (int k = 0; k < 4; k++) {
                A[j * 2 + 0][k] = x * P[8 + k] - P[0 + k];
                A[j * 2 + 1][k] = y * P[8 + k] - P[4 + k];
            }
        }
        /* _SVDcompute: m >= n -> temp_a = transpose(A) */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < m; r++) At[c * m + r] = A[r][c];
        orc_jacobi_svd(At, m, 4, NULL, Vt);
        for (int k = 0; k < 4; k++) {
            out4[k * n + i] = (float)Vt[12 + k];
            if (out4_f64) out4_f64[k * n + i] = Vt[12 + k];
        }
    }
}

/* icvTriangulatePoints with CV_64F points: the same fp64 A from double x, y; points4D is
 * CV_64F (the points' type), so the null vector is stored unrounded. */
void orc_triangulate_nview_f64(const double* Ps, int nv, const double* xs, int64_t n, double* out4)
{
    double At[4 * 32], Vt[16];
    const int m = 2 * nv;
    for (int64_t i = 0; i < n; i++) {
        double A[32][4];
        for (int j = 0; j < nv; j++) {
            const double* P = Ps + 12 * j;
            double x = xs[(j * n + i) * 2 + 0];
            double y = xs[(j * n + i) * 2 + 1];
            for (int k = 0; k < 4; k++) {
                A[j * 2 + 0][k] = x * P[8 + k] - P[0 + k];
                A[j * 2 + 1][k] = y * P[8 + k] - P[4 + k];
            }
        }
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < m; r++) At[c * m + r] = A[r][c];
        orc_jacobi_svd(At, m, 4, NULL, Vt);
        for (int k = 0; k < 4; k++) out4[k * n + i] = Vt[12 + k];
    }
}

/* ---- fundam.cpp convertPointsFromHomogeneous, f64, 4 -> 3 (scale = w != 0 ? 1./w : 1.) */
void orc_from_homogeneous_f64(const double* in, int64_t n, double* out)
{
    for (int64_t i = 0; i < n; i++) {
        double w = in[4 * i + 3];
        double scale = w != 0. ? 1. / w : 1.;
        out[3 * i + 0] = in[4 * i + 0] * scale;
        out[3 * i + 1] = in[4 * i + 1] * scale;
        out[3 * i + 2] = in[4 * i + 2] * scale;
    }
}

/* ---- fundam.cpp convertPointsFromHomogeneous, f32, 4 -> 3 --------------- */
/* in: n x 4 f32 (rows), out: n x 3 f32. */
void orc_from_homogeneous_f32(const float* in, int64_t n, float* out)
{
    for (int64_t i = 0; i < n; i++) {
        float w = in[4 * i + 3];
        float scale = w != 0.f ? 1.f / w : 1.f;
        out[3 * i + 0] = in[4 * i + 0] * scale;
        out[3 * i + 1] = in[4 * i + 1] * scale;
        out[3 * i + 2] = in[4 * i + 2] * scale;
    }
}
