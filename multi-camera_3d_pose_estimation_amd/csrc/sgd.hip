// Reprojection-error trajectory refinement for gfx950 — one workgroup per trajectory,
// the whole optimisation in one launch.
//
// Replaces Optimized_3d_Pose_Estimation.sgd_optimize (reference
// pose_refinement.py:894-1096, trajectory-only path run by the CLI at :1210-1214).
// Per overlapping window (create_batch_indices, :786-796) and per iteration:
//   pass A  forward costs   likelihood  0.5·dᵀΣ⁻¹d of every camera's projection
//                                       (project_points_torch :94-179) against the
//                                       camera-0 Gaussian (:863-889, quirk F7),
//                                       nan_mean (:221-229);
//                           smoothness  λs·mean‖x_t − 2x_{t−1} + x_{t−2}‖² (:836-845);
//                           body length λb·‖a − μb‖²/‖a‖², μ = a·b/b·b (:848-860)
//           + the likelihood gradient through the projection Jacobian (radial +
//           tangential distortion), unscaled, into a per-point buffer
//   pass B  scale it by 1/n and add the stencil and segment-length adjoints,
//           pulled per owned point; ‖g‖₂ for clip_grad_norm_ (:1045)
//   pass C  Adam over the WHOLE trajectory (torch single-tensor Adam; rows outside
//           the window keep moving with their momentum)
// then the reference's running-mean early stop, where the cost list doubles as
// the running-mean list (:987, :1070-1089, quirk F6), and the best snapshot.
//
// Rounding follows torch's f32 op order (contraction off); reductions are
// fp64 — results agree with the reference to f32 rounding, not bit-for-bit
// (its BLAS/pairwise summation order is not reproducible here).
#pragma clang fp contract(off)

#include "mvp_common.h"

#include <cmath>

namespace {

constexpr int kMaxSgdCams = 16;
constexpr int kMaxSeg = 32;
constexpr int kMaxJ = 64;
constexpr int kMaxJointSeg = 6;  // segments per joint listed for pass B (more: the full segment loop)
constexpr int kMaxLearn = 2;   // learnable cameras (joint trajectory + extrinsic branch)
constexpr int kCamGrad = 12;   // dR (9, row-major) + dT (3) per learnable camera

struct SgdArgs {
    const float* gauss;
    const float* traj0;
    const float* cams;
    const int* seg;
    const float* seg_len;
    float* ws;
    float* final_traj;
    float* best_traj;
    float* batch_costs;
    float* iter_means;
    int* iters;
    int T, V, J, n_seg;
    int B, stride, n_win;
    int traj_in_lds;
    mvp_sgd_params p;
    int n_learn;               // joint branch: cameras whose R, T are learnable (0 = trajectory only)
    int learn[kMaxLearn];
    float* cams_final;         // [M][n_learn][12]
    float* cams_best;          // [M][n_learn][12]
};

// The projection and its adjoint are templates over the lane's value type: float (one point)
// or f2v (two points per lane, the trajectory-only pass A): every operation is the same in the
// same order, so the two-point form issues v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32 — one
// instruction for both points, the same roundings (contraction stays off) — where the one-point
// form issues two.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float rcp_v(float b) { return __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ f2v rcp_v(f2v b) { return f2v{__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)}; }
__device__ __forceinline__ float fma_v(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ f2v fma_v(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

template <class V>
struct ProjT {
    V u, v;                     // pixel
    V x, y;                     // normalised (undistorted) coordinates
    V P2;                       // camera-frame depth
    V r2, rad, h2;
    V xd, yd;
};
using Proj = ProjT<float>;

// (a0 / b, a1 / b) for finite normal operands: one v_rcp_f32 and a Markstein correction
// step per quotient (q = a·r, e = a − q·b, q + e·r): the correctly rounded quotient except in
// rare double-rounding cases (≤ 1 ulp), 4 VALU operations against ~10 for the IEEE sequence.
// Range: v_rcp_f32 flushes for |b| < 2^-126 (a point within 1e-38 cm of the camera plane:
// here NaN; in torch x = P0 / P2 is ~1e30 or more, whose square overflows f32 in the
// distortion polynomial, so the term is non-finite there too and nan_mean's mask drops it in
// both — they differ only for a point within ~1e-38 cm of the camera centre itself) and
// returns 0 for |b| > 2^126, a camera-frame depth beyond 8.5e37 cm.  torch returns a / b there:
// ~0 for a moderate |a|, but O(1) when |a| is as large (a point ~1e38 cm away along any ray), so
// a trajectory that has diverged to the f32 overflow scale projects to the principal point here
// and to its true direction in torch — the two costs differ for such a point.  Every trajectory
// the reference's own runs produce stays many orders of magnitude inside that range; a per-lane
// range guard with an IEEE fallback measured +4.5-8 % per SGD iteration
// (profiles/r04_sgd_guard_ab.txt), so there is none.
template <class V>
__device__ __forceinline__ void div2_fast(V a0, V a1, V b, V& q0, V& q1) {
    const V r = rcp_v(b);
    const V p0 = a0 * r, p1 = a1 * r;
    q0 = fma_v(fma_v(-p0, b, a0), r, p0);
    q1 = fma_v(fma_v(-p1, b, a1), r, p1);
}

// project_points_torch (pose_refinement.py:118-177) for one point, torch op order.  kstd: K's
// last row is (0, 0, 1) (camera-uniform), so h2 = xd·0 + yd·0 + 1 is exactly 1 for finite xd, yd
// and u = h0 / 1 = h0: the division is skipped with identical results (a non-finite xd or yd
// gives a non-finite cost either way, which the likelihood's finite mask drops).
template <class V>
__device__ __forceinline__ ProjT<V> project(const float* __restrict__ c, V X0, V X1, V X2, bool ign, bool kstd) {
    const float* K = c;
    const float* R = c + 9;
    const float* T = c + 18;
    const float* d = c + 21;
    ProjT<V> o;
    const V P0 = X0 * R[0] + X1 * R[1] + X2 * R[2] + T[0];
    const V P1 = X0 * R[3] + X1 * R[4] + X2 * R[5] + T[1];
    const V P2 = X0 * R[6] + X1 * R[7] + X2 * R[8] + T[2];
    o.P2 = P2;
    div2_fast(P0, P1, P2, o.x, o.y);
    if (!ign) {
        const V x = o.x, y = o.y;
        const V r2 = x * x + y * y;
        const float k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3], k3 = d[4];
        const V rad = 1.f + k1 * r2 + k2 * (r2 * r2) + k3 * (r2 * r2 * r2);
        V xd = x * rad, yd = y * rad;
        xd = xd + (2.f * p1 * x * y + p2 * (r2 + 2.f * (x * x)));
        yd = yd + (p1 * (r2 + 2.f * (y * y)) + 2.f * p2 * x * y);
        o.r2 = r2;
        o.rad = rad;
        o.xd = xd;
        o.yd = yd;
    } else {
        o.r2 = V(0.f);
        o.rad = V(1.f);
        o.xd = o.x;
        o.yd = o.y;
    }
    const V h0 = o.xd * K[0] + o.yd * K[1] + K[2];
    const V h1 = o.xd * K[3] + o.yd * K[4] + K[5];
    if (kstd) {
        o.h2 = V(1.f);
        o.u = h0;
        o.v = h1;
    } else {
        const V h2 = o.xd * K[6] + o.yd * K[7] + K[8];
        o.h2 = h2;
        div2_fast(h0, h1, h2, o.u, o.v);
    }
    return o;
}

// d(u,v)/dX transposed applied to (gu, gv): the adjoint of project().
template <class V>
__device__ __forceinline__ void project_adjoint(const float* __restrict__ c, const ProjT<V>& o, bool ign, bool kstd,
                                                V gu, V gv, V& g0, V& g1, V& g2, V (&dP)[3]) {
    const float* K = c;
    const float* R = c + 9;
    const float* d = c + 21;
    // (u, v) = (h0, h1) / h2, h = K·[xd, yd, 1].  The adjoint's reciprocals are v_rcp_f32
    // (1 ulp): only the forward value needs torch's correctly rounded divisions, the gradient
    // already differs from autograd's by f32 summation order (an IEEE 1/x is ~10 VALU ops)
    V gxd, gyd;
    if (kstd) {  // K6 = K7 = 0, h2 = 1: the same values without the zero terms
        gxd = K[0] * gu + K[3] * gv;
        gyd = K[1] * gu + K[4] * gv;
    } else {
        const V ih2 = rcp_v(o.h2);
        gxd = ((K[0] - o.u * K[6]) * gu + (K[3] - o.v * K[6]) * gv) * ih2;
        gyd = ((K[1] - o.u * K[7]) * gu + (K[4] - o.v * K[7]) * gv) * ih2;
    }
    V gx = gxd, gy = gyd;
    if (!ign) {
        const V x = o.x, y = o.y, r2 = o.r2, rad = o.rad;
        const float k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3], k3 = d[4];
        const V drad = k1 + 2.f * k2 * r2 + 3.f * k3 * r2 * r2;
        const V dxx = rad + 2.f * x * x * drad + 2.f * p1 * y + 6.f * p2 * x;
        const V dxy = 2.f * x * y * drad + 2.f * p1 * x + 2.f * p2 * y;
        const V dyy = rad + 2.f * y * y * drad + 6.f * p1 * y + 2.f * p2 * x;
        gx = dxx * gxd + dxy * gyd;   // d(xd,yd)/dx is symmetric in its off-diagonal
        gy = dxy * gxd + dyy * gyd;
    }
    // x = P0/P2, y = P1/P2, P = R·X + T
    const V iP2 = rcp_v(o.P2);
    const V a = gx * iP2, b = gy * iP2, cz = -(gx * o.x + gy * o.y) * iP2;
    dP[0] = a;  // d/dP of the camera-frame point (the learnable extrinsics' chain)
    dP[1] = b;
    dP[2] = cz;
    g0 = R[0] * a + R[3] * b + R[6] * cz;
    g1 = R[1] * a + R[4] * b + R[7] * cz;
    g2 = R[2] * a + R[5] * b + R[8] * cz;
}

// Σ⁻¹ of (cov + 1e-6·I) (pose_refinement.py:663-668), cov = [g2 g3; g4 g5].
__device__ __forceinline__ void cov_inverse(const float* __restrict__ g, float& a00, float& a01, float& a10,
                                            float& a11) {
    const float c00 = g[2] + 1e-6f, c01 = g[3], c10 = g[4], c11 = g[5] + 1e-6f;
    const float det = c00 * c11 - c01 * c10;
    a00 = c11 / det;
    a01 = -c01 / det;
    a10 = -c10 / det;
    a11 = c00 / det;
}

// Per (frame, camera, joint): the Gaussian mean and Σ⁻¹, computed once per launch.
struct Target {
    float m0, m1, a00, a01, a10, a11;
};

__device__ __forceinline__ Target load_target(const float* __restrict__ tg) {
    const float2 p = *reinterpret_cast<const float2*>(tg);
    const float2 q = *reinterpret_cast<const float2*>(tg + 2);
    const float2 r = *reinterpret_cast<const float2*>(tg + 4);
    return {p.x, p.y, q.x, q.y, r.x, r.y};
}

// 0.5·dᵀΣ⁻¹d (the negated gaussian_likelihood quadratic term, :741-758)
__device__ __forceinline__ float quad_cost(const Target& g, float d0, float d1) {
    return 0.5f * ((d0 * g.a00 + d1 * g.a10) * d0 + (d0 * g.a01 + d1 * g.a11) * d1);
}

// points per thread in flight (independent loads issued together): 4 in the 256-thread
// workgroups (one wave per SIMD, ILP hides the latency); 1 in the 1,024-thread config-5 kernel,
// whose 4 waves per SIMD need <= 128 VGPRs (kU = 4 spills there; kU = 1 and 2 ran level:
// profiles/r04_sgd_occupancy_ab.txt)
template <int BS>
constexpr int points_in_flight() { return BS >= 1024 ? 1 : 4; }

constexpr int kRedCols = 2 * kCamGrad;  // widest block reduction: both learnable cameras' gradients

template <int BS, int NV, int NC>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (*red)[NC]) {
    static_assert(NV <= NC, "block_sum width");
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[i] += __shfl_xor(v[i], off, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0)
#pragma unroll
        for (int i = 0; i < NV; i++) red[w][i] = v[i];
    __syncthreads();
    // wave partials added in wave order; the k loop stays rolled, so only NV sums are live
    // (unrolled, the compiler loaded all BS / 64 x NV partials at once: 96 VGPRs at BS = 1,024)
    double s[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) s[i] = 0.0;
#pragma unroll 1
    for (int k = 0; k < BS / 64; k++)
#pragma unroll
        for (int i = 0; i < NV; i++) s[i] += red[k][i];
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = s[i];
}

__device__ __forceinline__ bool finite(float x) { return !(isnan(x) || isinf(x)); }

// (q / d, q % d) for 0 <= q < 2^24 and d >= 1 with rd = 1.f / d: the f32 product is within one
// of the quotient, and one correction step each way makes it exact (the integer division
// expands to ~25 VALU instructions, this to ~8)
__device__ __forceinline__ void divmod_small(int q, int d, float rd, int& quo, int& rem) {
    int i = (int)((float)q * rd);
    int r = q - i * d;
    if (r < 0) {
        i--;
        r += d;
    }
    if (r >= d) {
        i++;
        r -= d;
    }
    quo = i;
    rem = r;
}

// XL: the trajectory lives in LDS (T·J·3 floats within the LDS budget).  A template parameter,
// not a runtime pointer choice: through a pointer that may be either, every trajectory access
// compiles to a FLAT instruction (the vector-memory path, waits on both counters) instead of
// ds_read / ds_write.
template <int BS, bool LEARN, bool XL>
__global__ __launch_bounds__(BS) void sgd_kernel(SgdArgs a) {
    extern __shared__ float lds_traj[];
    __shared__ float cam_s[kMaxSgdCams * MVP_SGD_CAM_FLOATS];
    __shared__ int seg_s[kMaxSeg * 2];
    __shared__ float seglen_s[kMaxSeg];
    __shared__ int jseg[kMaxJ][kMaxJointSeg];  // per joint: the segments touching it, in segment order
    __shared__ int jseg_n[kMaxJ];
    __shared__ int jseg_over;
    __shared__ double red_s[BS / 64][kRedCols];
    __shared__ int learn_slot[kMaxSgdCams];            // camera -> learnable index, -1 = fixed
    __shared__ int cam_kstd[kMaxSgdCams];              // K's last row is (0, 0, 1)
    __shared__ float cstate[kMaxLearn * 2 * kCamGrad];  // Adam m | v of the learnable R, T
    __shared__ float cgrad[kMaxLearn * kCamGrad];       // the window's reduced camera gradient

    constexpr int kU = points_in_flight<BS>();
    const int m = blockIdx.x, tid = threadIdx.x;
    const int T = a.T, V = a.V, J = a.J, B = a.B, NS = a.n_seg;
    const int TJ = T * J, n3 = TJ * 3;
    const float rJ = 1.f / (float)J, rB = 1.f / (float)B;
    const bool ign = a.p.ignore_distortions != 0;
    const bool own = a.p.own_camera_gaussians != 0;
    const bool use_s = a.p.lambda_smooth > 0, use_b = a.p.lambda_body_length > 0;
    const float lam_s = (float)a.p.lambda_smooth, lam_b = (float)a.p.lambda_body_length;

    const int Vg = own ? V : 1;                     // cameras with their own Gaussian
    float* ws = a.ws + (size_t)m * ((size_t)4 * n3 + T + (size_t)T * V * J * 6);
    float* X = XL ? lds_traj : ws;
    float* mo = ws + n3;
    float* ve = ws + 2 * (size_t)n3;
    float* gb = ws + 3 * (size_t)n3;
    float* sterm = XL ? lds_traj + n3 : ws + 4 * (size_t)n3;  // per-window smoothness terms ‖D‖²
    float* tgt = ws + 4 * (size_t)n3 + T;           // [T][Vg][J][6] Target records
    const float* G = a.gauss + (size_t)m * T * V * J * 6;
    const float* X0 = a.traj0 + (size_t)m * n3;
    float* best = a.best_traj + (size_t)m * n3;

    for (int i = tid; i < V * MVP_SGD_CAM_FLOATS; i += BS) cam_s[i] = a.cams[i];
    const int NL = LEARN ? a.n_learn : 0;  // LEARN = false: the trajectory-only kernel, unchanged
    for (int c = tid; c < V; c += BS) {
        const float* K = a.cams + c * MVP_SGD_CAM_FLOATS;
        cam_kstd[c] = K[6] == 0.f && K[7] == 0.f && K[8] == 1.f;
        int sl = -1;
        for (int l = 0; l < NL; l++)
            if (a.learn[l] == c) sl = l;
        learn_slot[c] = sl;
    }
    for (int i = tid; i < kMaxLearn * 2 * kCamGrad; i += BS) cstate[i] = 0.f;
    for (int i = tid; i < NS; i += BS) {
        seg_s[2 * i] = a.seg[2 * i];
        seg_s[2 * i + 1] = a.seg[2 * i + 1];
        seglen_s[i] = a.seg_len[i];
    }
    if (tid == 0) jseg_over = 0;
    __syncthreads();
    for (int j = tid; j < J; j += BS) {
        int c = 0;
        for (int sg = 0; sg < NS; sg++)
            if (a.seg[2 * sg] == j || a.seg[2 * sg + 1] == j) {
                if (c < kMaxJointSeg) jseg[j][c] = sg;
                c++;
            }
        jseg_n[j] = c;
        if (c > kMaxJointSeg) jseg_over = 1;
    }
    for (int r = tid; r < T * Vg * J; r += BS) {
        const int j = r % J, tc = r / J, c = tc % Vg, t = tc / Vg;
        const float* g = G + (((size_t)t * V + c) * J + j) * 6;
        float A00, A01, A10, A11;
        cov_inverse(g, A00, A01, A10, A11);
        float* o = tgt + (size_t)r * 6;
        o[0] = g[0];
        o[1] = g[1];
        o[2] = A00;
        o[3] = A01;
        o[4] = A10;
        o[5] = A11;
    }
    for (int e = tid; e < n3; e += BS) {
        X[e] = X0[e];
        mo[e] = 0.f;
        ve[e] = 0.f;
        best[e] = __builtin_nanf("");
    }
    __syncthreads();

    // ‖a‖² of the repeated body-length vector (create_body_length_vect, :765-781)
    double aa = 0.0;
    for (int s = 0; s < NS; s++) aa += (double)seglen_s[s] * seglen_s[s];
    aa *= B;

    const float w1 = (float)(1.0 - a.p.beta1);
    const float b2 = (float)a.p.beta2, w2 = (float)(1.0 - a.p.beta2);
    const float eps = (float)a.p.adam_eps;
    const int n_win = a.n_win;

    double hist_sum[MVP_SGD_N_COSTS] = {0, 0, 0, 0};
    long hist_cnt = 0;
    float best_total = INFINITY;
    int no_imp = 0, it = 0, step = 0;

    while (no_imp < a.p.patience && it <= a.p.max_iter) {
        for (int w = 0; w < n_win; w++) {
            const int t0 = w * a.stride;
            const int nq = B * J;
            // ---- pass A: forward costs
            double acc[6] = {0, 0, 0, 0, 0, 0};   // lsum, lcnt, ssum, scnt, ab, bb
            float cg0[LEARN ? kCamGrad : 1], cg1[LEARN ? kCamGrad : 1];  // learnable cameras 0, 1: dR, dT
            if constexpr (LEARN)
#pragma unroll
                for (int k = 0; k < kCamGrad; k++) cg0[k] = cg1[k] = 0.f;
            // likelihood value AND its (not yet 1/n-scaled) gradient: one projection per
            // (point, camera) per step; the scale needs the global finite count.
            if constexpr (!LEARN && kU == 1) {
                // two points per lane (q0 and q0 + BS, the order the one-point loop visits them
                // in, so every sum is the same): the projection and its adjoint on f2v, packed
                // VALU instructions for both points
                for (int q0 = tid; q0 < nq; q0 += 2 * BS) {
                    const bool hb = q0 + BS < nq;
                    const int qa = q0, qb = hb ? q0 + BS : q0;
                    int ia, ja, ib, jb;
                    divmod_small(qa, J, rJ, ia, ja);
                    divmod_small(qb, J, rJ, ib, jb);
                    const int ta = t0 + ia, tb = t0 + ib;
                    const float* pa = X + 3 * (ta * J + ja);
                    const float* pb = X + 3 * (tb * J + jb);
                    const f2v X0 = {pa[0], pb[0]}, X1 = {pa[1], pb[1]}, X2 = {pa[2], pb[2]};
                    const Target tga = load_target(tgt + ((size_t)ta * Vg * J + ja) * 6);
                    const Target tgb = load_target(tgt + ((size_t)tb * Vg * J + jb) * 6);
                    float lsa = 0.f, lsb = 0.f;
                    int lca = 0, lcb = 0;
                    f2v g0 = {0.f, 0.f}, g1 = {0.f, 0.f}, g2 = {0.f, 0.f};
                    for (int c = 0; c < V; c++) {
                        const float* cam = cam_s + c * MVP_SGD_CAM_FLOATS;
                        const bool kstd = cam_kstd[c] != 0;  // camera-uniform
                        const ProjT<f2v> o = project(cam, X0, X1, X2, ign, kstd);
                        const Target gA = own ? load_target(tgt + (((size_t)ta * Vg + c) * J + ja) * 6) : tga;
                        const Target gB = own ? load_target(tgt + (((size_t)tb * Vg + c) * J + jb) * 6) : tgb;
                        const f2v a00 = {gA.a00, gB.a00}, a01 = {gA.a01, gB.a01};
                        const f2v a10 = {gA.a10, gB.a10}, a11 = {gA.a11, gB.a11};
                        const f2v d0 = o.u - f2v{gA.m0, gB.m0}, d1 = o.v - f2v{gA.m1, gB.m1};
                        const f2v val = 0.5f * ((d0 * a00 + d1 * a10) * d0 + (d0 * a01 + d1 * a11) * d1);
                        const bool fa = finite(val.x), fb = finite(val.y);
                        if (!fa && !fb) continue;
                        const f2v s01 = a01 + a10;
                        const f2v gu = 0.5f * (2.f * a00 * d0 + s01 * d1);
                        const f2v gv = 0.5f * (s01 * d0 + 2.f * a11 * d1);
                        f2v h0, h1, h2, dP[3];
                        project_adjoint(cam, o, ign, kstd, gu, gv, h0, h1, h2, dP);
                        if (fa && fb) {
                            lsa += val.x;
                            lsb += val.y;
                            lca++;
                            lcb++;
                            g0 += h0;
                            g1 += h1;
                            g2 += h2;
                        } else if (fa) {
                            lsa += val.x;
                            lca++;
                            g0.x += h0.x;
                            g1.x += h1.x;
                            g2.x += h2.x;
                        } else {
                            lsb += val.y;
                            lcb++;
                            g0.y += h0.y;
                            g1.y += h1.y;
                            g2.y += h2.y;
                        }
                    }
                    acc[0] += lsa;
                    acc[1] += lca;
                    gb[3 * qa + 0] = g0.x;
                    gb[3 * qa + 1] = g1.x;
                    gb[3 * qa + 2] = g2.x;
                    if (hb) {
                        acc[0] += lsb;
                        acc[1] += lcb;
                        gb[3 * qb + 0] = g0.y;
                        gb[3 * qb + 1] = g1.y;
                        gb[3 * qb + 2] = g2.y;
                    }
                }
            } else
            for (int q0 = tid; q0 < nq; q0 += kU * BS) {
                float xs[kU][3];
                Target tg[kU];
                int tq[kU], jq[kU];
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    const int q = min(q0 + u * BS, nq - 1);
                    int qi;
                    divmod_small(q, J, rJ, qi, jq[u]);
                    tq[u] = t0 + qi;
                    const float* x = X + 3 * (tq[u] * J + jq[u]);
                    xs[u][0] = x[0];
                    xs[u][1] = x[1];
                    xs[u][2] = x[2];
                    tg[u] = load_target(tgt + ((size_t)tq[u] * Vg * J + jq[u]) * 6);
                }
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    const int q = q0 + u * BS;
                    if (q >= nq) break;
                    float lsum = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
                    int lcnt = 0;
                    for (int c = 0; c < V; c++) {
                        const float* cam = cam_s + c * MVP_SGD_CAM_FLOATS;
                        const bool kstd = cam_kstd[c] != 0;  // camera-uniform
                        const Proj o = project(cam, xs[u][0], xs[u][1], xs[u][2], ign, kstd);
                        const Target g =
                            own ? load_target(tgt + (((size_t)tq[u] * Vg + c) * J + jq[u]) * 6) : tg[u];
                        const float d0 = o.u - g.m0, d1 = o.v - g.m1;
                        const float val = quad_cost(g, d0, d1);
                        if (!finite(val)) continue;
                        lsum += val;
                        lcnt++;
                        const float s01 = g.a01 + g.a10;
                        const float gu = 0.5f * (2.f * g.a00 * d0 + s01 * d1);
                        const float gv = 0.5f * (s01 * d0 + 2.f * g.a11 * d1);
                        float h0, h1, h2, dP[3];
                        project_adjoint(cam, o, ign, kstd, gu, gv, h0, h1, h2, dP);
                        if constexpr (LEARN) {
                            const int ls = learn_slot[c];
                            auto add_cam = [&](float (&cg)[kCamGrad]) {  // dP/dR_ij = X_j, dP/dT_i = 1
#pragma unroll
                                for (int i = 0; i < 3; i++) {
#pragma unroll
                                    for (int jj = 0; jj < 3; jj++) cg[3 * i + jj] += dP[i] * xs[u][jj];
                                    cg[9 + i] += dP[i];
                                }
                            };
                            if (ls == 0)
                                add_cam(cg0);
                            else if (ls == 1)
                                add_cam(cg1);
                        }
                        g0 += h0;
                        g1 += h1;
                        g2 += h2;
                    }
                    acc[0] += lsum;
                    acc[1] += lcnt;
                    gb[3 * q + 0] = g0;
                    gb[3 * q + 1] = g1;
                    gb[3 * q + 2] = g2;
                }
            }
            if (use_s)
                for (int i = 2 + tid; i < B; i += BS) {
                    const int t = t0 + i;
                    const float* xa = X + 3 * t * J;
                    const float* xb = xa - 3 * J;
                    const float* xc = xb - 3 * J;
                    float ss = 0.f;
                    for (int e = 0; e < 3 * J; e++) {
                        const float D = (xa[e] - xb[e]) - (xb[e] - xc[e]);
                        ss += D * D;
                    }
                    const float nrm = sqrtf(ss);
                    const float term = nrm * nrm;
                    sterm[i] = term;
                    if (finite(term)) {
                        acc[2] += term;
                        acc[3] += 1.0;
                    }
                }
            if (use_b)
                for (int r = tid; r < NS * B; r += BS) {
                    int s, tr;
                    divmod_small(r, B, rB, s, tr);
                    const int t = t0 + tr;
                    const float* xa = X + 3 * (t * J + seg_s[2 * s]);
                    const float* xb = X + 3 * (t * J + seg_s[2 * s + 1]);
                    const float e0 = xb[0] - xa[0], e1 = xb[1] - xa[1], e2 = xb[2] - xa[2];
                    const float len = sqrtf(e0 * e0 + e1 * e1 + e2 * e2);
                    acc[4] += (double)seglen_s[s] * len;
                    acc[5] += (double)len * len;
                }
            block_sum<BS>(acc, red_s);
            if constexpr (LEARN) {  // the learnable cameras' gradient sums
                double cgd[kRedCols];
#pragma unroll
                for (int k = 0; k < kCamGrad; k++) {
                    cgd[k] = cg0[k];
                    cgd[kCamGrad + k] = cg1[k];
                }
                block_sum<BS>(cgd, red_s);
                const double sc = acc[1] > 0 ? 1.0 / acc[1] : 0.0;  // the likelihood's 1/n, as lscale
                if (tid == 0)
#pragma unroll
                    for (int k = 0; k < kRedCols; k++)
                        if (k < NL * kCamGrad) cgrad[k] = (float)(cgd[k] * sc);
                __syncthreads();
            }
            const float L = (float)(acc[0] / acc[1]);
            const float S = lam_s * (float)(acc[2] / acc[3]);
            const float mu = (float)acc[4] / (float)acc[5];
            const float lscale = acc[1] > 0 ? (float)(1.0 / acc[1]) : 0.f;
            const float sscale = acc[3] > 0 ? 2.f * lam_s * (float)(1.0 / acc[3]) : 0.f;
            const float bscale = -2.f * lam_b * mu / (float)aa;

            // ---- pass B: gradient of the window's total cost, pulled per owned point
            double acc2[2] = {0, 0};   // ‖g‖², Σ r²
            for (int q = tid; q < nq; q += BS) {
                int i, j;
                divmod_small(q, J, rJ, i, j);
                const int t = t0 + i;
                float g0 = gb[3 * q + 0] * lscale, g1 = gb[3 * q + 1] * lscale, g2 = gb[3 * q + 2] * lscale;
                if (use_s) {
                    // terms centred at t (coef +1), t+1 (-2), t+2 (+1), each 2·λs/n·D
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const int ic = i + k;
                        if (ic < 2 || ic >= B || !finite(sterm[ic])) continue;
                        const float coef = (k == 1 ? -2.f : 1.f) * sscale;
                        const float* xa = X + 3 * ((t + k) * J + j);
                        const float* xb = xa - 3 * J;
                        const float* xc = xb - 3 * J;
                        g0 += coef * ((xa[0] - xb[0]) - (xb[0] - xc[0]));
                        g1 += coef * ((xa[1] - xb[1]) - (xb[1] - xc[1]));
                        g2 += coef * ((xa[2] - xb[2]) - (xb[2] - xc[2]));
                    }
                }
                if (use_b) {
                    // the segments touching joint j, in segment order (the same additions as the
                    // loop over all NS segments, which stays for a joint in more than kMaxJointSeg)
                    const int nsj = jseg_over ? NS : jseg_n[j];
                    for (int m = 0; m < nsj; m++) {
                        const int s = jseg_over ? m : jseg[j][m];
                        const int ja = seg_s[2 * s], jb = seg_s[2 * s + 1];
                        if (ja != j && jb != j) continue;
                        const float* xa = X + 3 * (t * J + ja);
                        const float* xb = X + 3 * (t * J + jb);
                        const float e0 = xb[0] - xa[0], e1 = xb[1] - xa[1], e2 = xb[2] - xa[2];
                        const float len = sqrtf(e0 * e0 + e1 * e1 + e2 * e2);
                        if (!(len > 0.f)) continue;
                        const float r = seglen_s[s] - mu * len;
                        float dl = bscale * r / len;
                        if (ja == j) dl = -dl;
                        if (ja == jb) dl = 0.f;
                        g0 += dl * e0;
                        g1 += dl * e1;
                        g2 += dl * e2;
                    }
                }
                gb[3 * q + 0] = g0;
                gb[3 * q + 1] = g1;
                gb[3 * q + 2] = g2;
                acc2[0] += (double)g0 * g0 + (double)g1 * g1 + (double)g2 * g2;
            }
            if (use_b)
                for (int r = tid; r < NS * B; r += BS) {
                    int s, tr;
                    divmod_small(r, B, rB, s, tr);
                    const int t = t0 + tr;
                    const float* xa = X + 3 * (t * J + seg_s[2 * s]);
                    const float* xb = X + 3 * (t * J + seg_s[2 * s + 1]);
                    const float e0 = xb[0] - xa[0], e1 = xb[1] - xa[1], e2 = xb[2] - xa[2];
                    const float len = sqrtf(e0 * e0 + e1 * e1 + e2 * e2);
                    const float rr = seglen_s[s] - mu * len;
                    acc2[1] += (double)rr * rr;
                }
            block_sum<BS>(acc2, red_s);
            float gnorm = (float)sqrt(acc2[0]);
            if (NL > 0) {
                // clip_grad_norm_ over [R_0, T_0, (R_1, T_1,) trajectory]: per-tensor norms, then
                // the norm of the norms
                double tot = (double)gnorm * gnorm;
                for (int l = 0; l < NL; l++) {
                    double r2 = 0.0, t2 = 0.0;
                    for (int k = 0; k < 9; k++) r2 += (double)cgrad[l * kCamGrad + k] * cgrad[l * kCamGrad + k];
                    for (int k = 9; k < kCamGrad; k++) t2 += (double)cgrad[l * kCamGrad + k] * cgrad[l * kCamGrad + k];
                    const float nr = (float)sqrt(r2), nt = (float)sqrt(t2);
                    tot += (double)nr * nr + (double)nt * nt;
                }
                gnorm = (float)sqrt(tot);
            }
            const float coef = fminf((float)a.p.max_grad_norm / (gnorm + 1e-6f), 1.f);
            const float Bc = lam_b * (float)acc2[1] / (float)aa;

            // ---- pass C: Adam over the whole trajectory (torch _single_tensor_adam)
            step++;
            const double bc1 = 1.0 - pow(a.p.beta1, (double)step);
            const double bc2 = 1.0 - pow(a.p.beta2, (double)step);
            const float nstep = (float)(-(a.p.lr / bc1));
            const float bc2s = (float)sqrt(bc2);
            const int wlo = t0 * J * 3, whi = (t0 + B) * J * 3;
            if (tid < NL * kCamGrad) {  // the learnable R, T: same single-tensor Adam step
                const int l = tid / kCamGrad, k = tid - l * kCamGrad;
                float* prm = cam_s + a.learn[l] * MVP_SGD_CAM_FLOATS + (k < 9 ? 9 + k : 18 + (k - 9));
                const float g = cgrad[tid] * coef;
                float mv = cstate[tid];
                mv = (w1 < 0.5f) ? mv + w1 * (g - mv) : g - (g - mv) * (1.f - w1);
                float vv = cstate[NL * kCamGrad + tid] * b2;
                vv = vv + w2 * g * g;
                cstate[tid] = mv;
                cstate[NL * kCamGrad + tid] = vv;
                const float denom = sqrtf(vv) / bc2s + eps;
                *prm = *prm + nstep * mv / denom;
            }
            // kA coordinates per thread per round, every load issued before the first store
            // (the stores could alias the next coordinate's loads for the compiler)
            constexpr int kA = 4;
            for (int e0 = tid; e0 < n3; e0 += kA * BS) {
                float gg[kA], m0[kA], v0[kA], x0[kA];
#pragma unroll
                for (int u = 0; u < kA; u++) {
                    const int e = min(e0 + u * BS, n3 - 1);
                    gg[u] = (e >= wlo && e < whi) ? gb[e - wlo] : 0.f;
                    m0[u] = mo[e];
                    v0[u] = ve[e];
                    x0[u] = X[e];
                }
#pragma unroll
                for (int u = 0; u < kA; u++) {
                    const int e = e0 + u * BS;
                    if (e >= n3) break;
                    const float g = (e >= wlo && e < whi) ? gg[u] * coef : 0.f;
                    float mv = m0[u];
                    mv = (w1 < 0.5f) ? mv + w1 * (g - mv) : g - (g - mv) * (1.f - w1);
                    float vv = v0[u] * b2;
                    vv = vv + w2 * g * g;
                    mo[e] = mv;
                    ve[e] = vv;
                    const float denom = sqrtf(vv) / bc2s + eps;
                    X[e] = x0[u] + nstep * mv / denom;
                }
            }
            __syncthreads();

            float total = L;
            if (use_s) total = total + S;
            if (use_b) total = total + Bc;
            const float rec[MVP_SGD_N_COSTS] = {total, L, use_s ? S : 0.f, use_b ? Bc : 0.f};
#pragma unroll
            for (int k = 0; k < MVP_SGD_N_COSTS; k++) hist_sum[k] += rec[k];
            hist_cnt++;
            if (tid == 0) {
                float* bc = a.batch_costs + (((size_t)m * (a.p.max_iter + 1) + it) * n_win + w) * MVP_SGD_N_COSTS;
#pragma unroll
                for (int k = 0; k < MVP_SGD_N_COSTS; k++) bc[k] = rec[k];
            }
        }
        // running mean over the shared list (F6): append the mean to the same list
        float mean[MVP_SGD_N_COSTS];
#pragma unroll
        for (int k = 0; k < MVP_SGD_N_COSTS; k++) mean[k] = (float)(hist_sum[k] / (double)hist_cnt);
#pragma unroll
        for (int k = 0; k < MVP_SGD_N_COSTS; k++) hist_sum[k] += mean[k];
        hist_cnt++;
        if (tid == 0) {
            float* im = a.iter_means + ((size_t)m * (a.p.max_iter + 1) + it) * MVP_SGD_N_COSTS;
#pragma unroll
            for (int k = 0; k < MVP_SGD_N_COSTS; k++) im[k] = mean[k];
        }
        if (mean[0] < best_total - (float)a.p.tolerance) {
            best_total = mean[0];
            for (int e = tid; e < n3; e += BS) best[e] = X[e];
            if (tid < NL * kCamGrad) {
                const int l = tid / kCamGrad, k = tid - l * kCamGrad;
                a.cams_best[((size_t)m * NL + l) * kCamGrad + k] =
                    cam_s[a.learn[l] * MVP_SGD_CAM_FLOATS + (k < 9 ? 9 + k : 18 + (k - 9))];
            }
            no_imp = 0;
        } else {
            no_imp++;
        }
        it++;
        if (no_imp >= a.p.patience) break;
    }
    float* fin = a.final_traj + (size_t)m * n3;
    for (int e = tid; e < n3; e += BS) fin[e] = X[e];
    if (tid < NL * kCamGrad) {
        const int l = tid / kCamGrad, k = tid - l * kCamGrad;
        a.cams_final[((size_t)m * NL + l) * kCamGrad + k] =
            cam_s[a.learn[l] * MVP_SGD_CAM_FLOATS + (k < 9 ? 9 + k : 18 + (k - 9))];
    }
    if (tid == 0) a.iters[m] = it;
}

__global__ void project_kernel(const float* __restrict__ pts, long n, const float* __restrict__ cam, int ign,
                               float* __restrict__ uv) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c[MVP_SGD_CAM_FLOATS];
#pragma unroll
    for (int k = 0; k < MVP_SGD_CAM_FLOATS; k++) c[k] = cam[k];
    const Proj o = project(c, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], ign != 0, false);
    uv[2 * i] = o.u;
    uv[2 * i + 1] = o.v;
}

// ---- extrinsic-from-samples cost (pose_refinement.py:800-831): the learnable camera's
// reprojection of the triangulated Gaussian samples against the target Gaussians,
// cost = -nan_mean(-0.5 dᵀΣ⁻¹d) over (t, joint, sample), and its gradient with respect to
// the camera's R (3x3 matrix entries, the reference's default learnable form) and T.
// dcost/dP (camera-frame point) comes from the projection adjoint; dP/dR_ij = X_j,
// dP/dT_i = 1.  One grid-stride pass; per-block fp64 partial sums
// [quad sum, finite count, dR (9, row-major), dT (3)] — the host reduces and steps Adam.
constexpr int kExtBlock = 256;
constexpr int kExtSums = 14;

__global__ __launch_bounds__(kExtBlock) void extrinsic_grad_kernel(const float* __restrict__ samples,
                                                                   const float* __restrict__ tgt, int n_samples,
                                                                   long n_points, const float* __restrict__ cam,
                                                                   int ign, double* __restrict__ partial) {
    __shared__ double red[kExtBlock / 64][8];
    float c[MVP_SGD_CAM_FLOATS];
#pragma unroll
    for (int k = 0; k < MVP_SGD_CAM_FLOATS; k++) c[k] = cam[k];
    const float* K = c;
    double acc[kExtSums];
#pragma unroll
    for (int k = 0; k < kExtSums; k++) acc[k] = 0.0;
    for (long i = (long)blockIdx.x * kExtBlock + threadIdx.x; i < n_points; i += (long)gridDim.x * kExtBlock) {
        const float X0 = samples[3 * i], X1 = samples[3 * i + 1], X2 = samples[3 * i + 2];
        const Target g = load_target(tgt + (i / n_samples) * 6);
        const Proj o = project(c, X0, X1, X2, ign != 0, false);
        const float d0 = o.u - g.m0, d1 = o.v - g.m1;
        const float val = quad_cost(g, d0, d1);
        if (!finite(val)) continue;
        const float s01 = g.a01 + g.a10;
        const float gu = 0.5f * (2.f * g.a00 * d0 + s01 * d1);
        const float gv = 0.5f * (s01 * d0 + 2.f * g.a11 * d1);
        // project_adjoint up to the camera-frame point P = R X + T
        const float ih2 = 1.f / o.h2;
        const float gxd = ((K[0] - o.u * K[6]) * gu + (K[3] - o.v * K[6]) * gv) * ih2;
        const float gyd = ((K[1] - o.u * K[7]) * gu + (K[4] - o.v * K[7]) * gv) * ih2;
        float gx = gxd, gy = gyd;
        if (!ign) {
            const float* d = c + 21;
            const float x = o.x, y = o.y, r2 = o.r2, rad = o.rad;
            const float k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3], k3 = d[4];
            const float drad = k1 + 2.f * k2 * r2 + 3.f * k3 * r2 * r2;
            const float dxx = rad + 2.f * x * x * drad + 2.f * p1 * y + 6.f * p2 * x;
            const float dxy = 2.f * x * y * drad + 2.f * p1 * x + 2.f * p2 * y;
            const float dyy = rad + 2.f * y * y * drad + 6.f * p1 * y + 2.f * p2 * x;
            gx = dxx * gxd + dxy * gyd;
            gy = dxy * gxd + dyy * gyd;
        }
        const float iP2 = __builtin_amdgcn_rcpf(o.P2);
        const float gp[3] = {gx * iP2, gy * iP2, -(gx * o.x + gy * o.y) * iP2};
        const float xs[3] = {X0, X1, X2};
        acc[0] += val;
        acc[1] += 1.0;
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int q = 0; q < 3; q++) acc[2 + 3 * r + q] += (double)gp[r] * xs[q];
            acc[11 + r] += gp[r];
        }
    }
    // block reduction in two halves of 7 (red holds 8 per wave)
#pragma unroll
    for (int half = 0; half < 2; half++) {
        double v[7];
#pragma unroll
        for (int k = 0; k < 7; k++) v[k] = acc[7 * half + k];
        block_sum<kExtBlock, 7>(v, red);
        if (threadIdx.x == 0)
#pragma unroll
            for (int k = 0; k < 7; k++) partial[(long)blockIdx.x * kExtSums + 7 * half + k] = v[k];
        __syncthreads();
    }
}

// ---- one Adam step of the extrinsic-from-samples branch on the device (pose_refinement.py:
// 1039-1050 with the learnable R (3x3 matrix) and T): the partial sums of the pass above ->
// cost / gradient (f32 casts of the fp64 means, as the host path), clip_grad_norm_([R, T],
// 1.0) (per-tensor norms then the norm of norms, accumulated in fp64 and cast to f32, like
// ATen's CPU reduction), torch single-tensor Adam per tensor; the camera record the next pass
// reads is updated in place and the step's cost and parameters are appended to the history.
// One workgroup; state = [m (12) | v (12) | step (as float bits)].
constexpr int kAdamBlock = 256;

__global__ __launch_bounds__(kAdamBlock) void extrinsic_adam_kernel(const double* __restrict__ partial, int n_blocks,
                                                                    float* __restrict__ cam, float* __restrict__ state,
                                                                    double lr, double beta1, double beta2,
                                                                    double adam_eps, double max_norm,
                                                                    float* __restrict__ cost_hist,
                                                                    float* __restrict__ param_hist) {
    __shared__ double red[kAdamBlock / 64][8];
    __shared__ double sums[kExtSums];
#pragma unroll
    for (int half = 0; half < 2; half++) {
        double v[7];
#pragma unroll
        for (int k = 0; k < 7; k++) v[k] = 0.0;
        for (int b = threadIdx.x; b < n_blocks; b += kAdamBlock)
#pragma unroll
            for (int k = 0; k < 7; k++) v[k] += partial[(long)b * kExtSums + 7 * half + k];
        block_sum<kAdamBlock, 7>(v, red);
        if (threadIdx.x == 0)
#pragma unroll
            for (int k = 0; k < 7; k++) sums[7 * half + k] = v[k];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    int* stepp = reinterpret_cast<int*>(state + 24);
    const int step = *stepp + 1;
    *stepp = step;
    const double cnt = sums[1];
    float g[12];
#pragma unroll
    for (int k = 0; k < 12; k++) g[k] = (float)(sums[2 + k] / cnt);
    double nR = 0.0, nT = 0.0;
#pragma unroll
    for (int k = 0; k < 9; k++) nR += (double)g[k] * g[k];
#pragma unroll
    for (int k = 9; k < 12; k++) nT += (double)g[k] * g[k];
    const float fR = (float)sqrt(nR), fT = (float)sqrt(nT);
    const float total = (float)sqrt((double)fR * fR + (double)fT * fT);
    const float coef = fminf((float)max_norm / (total + 1e-6f), 1.f);
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2);
    const double bc1 = 1.0 - pow(beta1, (double)step), bc2 = 1.0 - pow(beta2, (double)step);
    const float nstep = (float)(-(lr / bc1));
    const float bc2s = (float)sqrt(bc2);
    const float eps = (float)adam_eps;
    float* m = state;
    float* vv = state + 12;
    // learnable values live in the camera record: R at [9, 18), T at [18, 21)
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const float gk = g[k] * coef;
        float mv = m[k];
        mv = (w1 < 0.5f) ? mv + w1 * (gk - mv) : gk - (gk - mv) * (1.f - w1);
        float ve = vv[k] * b2;
        ve = ve + w2 * gk * gk;
        m[k] = mv;
        vv[k] = ve;
        const float denom = sqrtf(ve) / bc2s + eps;
        cam[9 + k] = cam[9 + k] + nstep * mv / denom;
    }
    cost_hist[step - 1] = (float)(sums[0] / cnt);
#pragma unroll
    for (int k = 0; k < 12; k++) param_hist[(long)(step - 1) * 12 + k] = cam[9 + k];
}

}  // namespace

extern "C" int mvp_sgd_workspace_floats(int M, int T, int V, int J, int64_t* out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(out && M > 0 && T > 0 && V > 0 && J > 0, "mvp_sgd_workspace_floats: bad arguments");
    *out = (int64_t)M * ((int64_t)4 * T * J * 3 + T + (int64_t)T * V * J * 6);
    MVP_ABI_END
}

namespace {
void sgd_launch(const float* gauss, const float* traj0, const float* cams, int M, int T, int V, int J, const int* seg,
                const float* seg_len, int n_seg, const mvp_sgd_params* p, float* workspace, float* final_traj,
                float* best_traj, float* batch_costs, float* iter_means, int* iters, const int* learn, int n_learn,
                float* cams_final, float* cams_best, void* stream) {
    MVP_REQUIRE(p && gauss && traj0 && cams && workspace && final_traj && best_traj && batch_costs && iter_means &&
                    iters,
                "mvp_sgd_refine: null pointer");
    MVP_REQUIRE(M > 0 && T > 0 && V > 0 && J > 0, "mvp_sgd_refine: M, T, V, J must be positive");
    MVP_REQUIRE(V <= kMaxSgdCams, "mvp_sgd_refine: V=%d > %d cameras", V, kMaxSgdCams);
    MVP_REQUIRE(J <= kMaxJ, "mvp_sgd_refine: J=%d > %d joints", J, kMaxJ);
    MVP_REQUIRE((int64_t)T * J * 3 < (1 << 24), "mvp_sgd_refine: T*J*3 = %lld >= 2^24 coordinates",
                (long long)T * J * 3);  // divmod_small's exact range (and far past any real recording)
    MVP_REQUIRE(n_seg >= 0 && n_seg <= kMaxSeg, "mvp_sgd_refine: n_seg=%d outside [0, %d]", n_seg, kMaxSeg);
    MVP_REQUIRE(n_seg == 0 || (seg && seg_len), "mvp_sgd_refine: segments missing");
    MVP_REQUIRE(p->lambda_body_length <= 0 || n_seg > 0,
                "mvp_sgd_refine: lambda_body_length > 0 needs body lengths (reference create_body_length_vect)");
    MVP_REQUIRE(p->batch_size >= 2 && p->batch_size <= T, "mvp_sgd_refine: batch_size=%d outside [2, T=%d]",
                p->batch_size, T);
    MVP_REQUIRE(p->max_iter >= 0 && p->patience >= 0, "mvp_sgd_refine: max_iter/patience must be >= 0");
    SgdArgs a;
    a.gauss = gauss;
    a.traj0 = traj0;
    a.cams = cams;
    a.seg = seg;
    a.seg_len = seg_len;
    a.ws = workspace;
    a.final_traj = final_traj;
    a.best_traj = best_traj;
    a.batch_costs = batch_costs;
    a.iter_means = iter_means;
    a.iters = iters;
    a.T = T;
    a.V = V;
    a.J = J;
    a.n_seg = n_seg;
    a.B = p->batch_size;
    a.stride = p->batch_size / 2;
    // windows cover the first floor(T/B)*B rows (sgd_optimize :900-905); later rows only see Adam
    // with zero gradient, i.e. stay where they started.
    const int t_win = (T / a.B) * a.B;
    a.n_win = (t_win - a.B) / a.stride + 1;
    a.p = *p;
    MVP_REQUIRE(n_learn >= 0 && n_learn <= kMaxLearn, "mvp_sgd_refine_cams: n_learn=%d outside [0, %d]", n_learn,
                kMaxLearn);
    MVP_REQUIRE(n_learn == 0 || (learn && cams_final && cams_best), "mvp_sgd_refine_cams: null pointer");
    a.n_learn = n_learn;
    for (int l = 0; l < kMaxLearn; l++) a.learn[l] = l < n_learn ? learn[l] : -1;
    for (int l = 0; l < n_learn; l++) {
        MVP_REQUIRE(learn[l] >= 0 && learn[l] < V, "mvp_sgd_refine_cams: camera slot %d outside [0, V=%d)", learn[l], V);
        for (int q = 0; q < l; q++)
            MVP_REQUIRE(learn[q] != learn[l], "mvp_sgd_refine_cams: camera slot %d listed twice", learn[l]);
    }
    a.cams_final = cams_final;
    a.cams_best = cams_best;
    const size_t traj_bytes = ((size_t)T * J * 3 + T) * sizeof(float);  // trajectory + smoothness terms
    constexpr size_t kLdsBudget = 120 * 1024;
    a.traj_in_lds = traj_bytes <= kLdsBudget;
    const size_t lds = a.traj_in_lds ? traj_bytes : 0;
    hipStream_t s = (hipStream_t)stream;
    auto launch = [&](auto kern, int bs) {
        MVP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget));
        hipLaunchKernelGGL(kern, dim3(M), dim3(bs), lds, s, a);
    };
    if (n_learn > 0) {  // joint branch: one kernel width (the camera gradient's registers)
        if (a.traj_in_lds) launch(sgd_kernel<256, true, true>, 256);
        else launch(sgd_kernel<256, true, false>, 256);
    } else if (T * J > 1024) {  // 16 waves: 4 per SIMD (M = 256 config 5: 0.211 -> 0.170 ms per iteration vs 512)
        if (a.traj_in_lds) launch(sgd_kernel<1024, false, true>, 1024);
        else launch(sgd_kernel<1024, false, false>, 1024);
    } else {
        if (a.traj_in_lds) launch(sgd_kernel<256, false, true>, 256);
        else launch(sgd_kernel<256, false, false>, 256);
    }
    MVP_HIP(hipGetLastError());
}
}  // namespace

extern "C" int mvp_sgd_refine(const float* gauss, const float* traj0, const float* cams, int M, int T, int V, int J,
                              const int* seg, const float* seg_len, int n_seg, const mvp_sgd_params* p,
                              float* workspace, float* final_traj, float* best_traj, float* batch_costs,
                              float* iter_means, int* iters, void* stream) {
    MVP_ABI_BEGIN
    sgd_launch(gauss, traj0, cams, M, T, V, J, seg, seg_len, n_seg, p, workspace, final_traj, best_traj, batch_costs,
               iter_means, iters, nullptr, 0, nullptr, nullptr, stream);
    MVP_ABI_END
}

extern "C" int mvp_sgd_refine_cams(const float* gauss, const float* traj0, const float* cams, int M, int T, int V,
                                   int J, const int* seg, const float* seg_len, int n_seg, const mvp_sgd_params* p,
                                   float* workspace, float* final_traj, float* best_traj, float* batch_costs,
                                   float* iter_means, int* iters, const int* learn_cam_host, int n_learn,
                                   float* cams_final, float* cams_best, void* stream) {
    MVP_ABI_BEGIN
    sgd_launch(gauss, traj0, cams, M, T, V, J, seg, seg_len, n_seg, p, workspace, final_traj, best_traj, batch_costs,
               iter_means, iters, learn_cam_host, n_learn, cams_final, cams_best, stream);
    MVP_ABI_END
}

extern "C" int mvp_project_points(const float* pts, int64_t n, const float* cam, int ignore_distortions, float* uv,
                                  void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n >= 0 && (n == 0 || (pts && cam && uv)), "mvp_project_points: bad arguments");
    if (n == 0) return MVP_OK;
    constexpr int kBlock = 256;
    hipLaunchKernelGGL(project_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, pts, (long)n, cam, ignore_distortions, uv);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_extrinsic_sample_grad(const float* samples, const float* targets, int n_samples,
                                         int64_t n_points, const float* cam, int ignore_distortions, int n_blocks,
                                         double* partial, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n_samples > 0 && n_points >= 0 && n_points % n_samples == 0 && n_blocks > 0,
                "mvp_extrinsic_sample_grad: bad sizes");
    MVP_REQUIRE(samples && targets && cam && partial, "mvp_extrinsic_sample_grad: NULL device pointer");
    hipLaunchKernelGGL(extrinsic_grad_kernel, dim3((unsigned)n_blocks), dim3(kExtBlock), 0, (hipStream_t)stream,
                       samples, targets, n_samples, (long)n_points, cam, ignore_distortions, partial);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}

extern "C" int mvp_extrinsic_adam_step(const double* partial, int n_blocks, float* cam, float* state, double lr,
                                       double beta1, double beta2, double adam_eps, double max_norm,
                                       float* cost_hist, float* param_hist, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n_blocks > 0 && partial && cam && state && cost_hist && param_hist,
                "mvp_extrinsic_adam_step: bad arguments");
    hipLaunchKernelGGL(extrinsic_adam_kernel, dim3(1), dim3(kAdamBlock), 0, (hipStream_t)stream, partial, n_blocks,
                       cam, state, lr, beta1, beta2, adam_eps, max_norm, cost_hist, param_hist);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}
