/*
 * mvpose.h — C-ABI of libmvpose.so, the MI355X-native (gfx950) multi-view 3D
 * pose hot path.  Drop-in boundary for the reference's per-frame
 * 2D-detect -> DLT-triangulate loop and its reprojection SGD
 * (sashapersonxyz/Multi-camera_3D_Pose_Estimation).
 *
 * Conventions
 *   - Every pointer named *_dev is a DEVICE pointer owned by the caller
 *     (e.g. a torch tensor's data_ptr()).  Pointers named *_host are host
 *     memory read synchronously during the call.
 *   - Every compute call takes a stream (a hipStream_t passed as void*; NULL =
 *     the default stream) and is asynchronous, stream-ordered work.
 *   - Every function returns int: MVP_OK (0) or a negative MVP_ERR_* code; it
 *     never throws across the ABI.  mvp_last_error() returns the message of the
 *     calling thread's last failure.
 *   - Handles may be used from one thread at a time; distinct handles/streams
 *     are independent.
 *   - No torch, numpy or C++ types cross this boundary.
 */
#ifndef MVPOSE_H
#define MVPOSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVP_ABI_VERSION 1

#define MVP_OK 0
#define MVP_ERR_ARG (-1)      /* invalid argument / shape */
#define MVP_ERR_HIP (-2)      /* HIP runtime error */
#define MVP_ERR_NOMEM (-3)    /* allocation failure */
#define MVP_ERR_INTERNAL (-4) /* unexpected internal failure */

int mvp_abi_version(void);
const char* mvp_last_error(void);

/* ---------------------------------------------------------------------------
 * Camera parameter block: one MVP_CAM_DOUBLES-double record per camera,
 *   [ K(3x3 row-major) | dist(k1,k2,p1,p2,k3) | R(3x3) | T(3) | P = K[R|T] (3x4) | pad(2) ]
 * K/dist/R/T are utils.get_params_from_name's values (reference utils.py:807-828);
 * P is computed by the caller exactly as utils.py:1318-1319 does (np.dot, fp64),
 * or with mvp_camera_pack.
 * ------------------------------------------------------------------------- */
#define MVP_CAM_DOUBLES 40

/* Host helper: pack one camera record (P = K·[R|T] in fp64, row-major loops). */
int mvp_camera_pack(const double* K_host, const double* dist5_host, const double* R_host,
                    const double* T_host, double* out_record_host);

/* ---------------------------------------------------------------------------
 * Triangulation (replaces pose_estimation.get_pose_3D, pose_estimation.py:11-65,
 * and its T*J calls of utils.triangulate_points, utils.py:1277-1336, i.e.
 * cv.undistortPoints x2 + cv.triangulatePoints + cv.convertPointsFromHomogeneous).
 *
 * kpts_dev : [n_points][3][V] float32 — the reference kpts_2d layout (T,J,3,V)
 *            flattened over (T,J); rows are x, y, confidence.
 * cams_dev : [n_cams][MVP_CAM_DOUBLES] float64.
 * cam_idx_host / n_cam_idx : camera_indices (reference hard-codes [0,1],
 *            pose_estimation.py:319); 2 <= n_cam_idx <= 8, each < min(V, n_cams).
 * mode     : MVP_TRI_REFERENCE — per point, the two highest-confidence listed
 *              cameras in ASCENDING confidence order (np.argsort(conf)[-2:],
 *              pose_estimation.py:36), parameters keyed by selection position
 *              (pose_estimation.py:44-45), OpenCV 4.9 numerics;
 *            MVP_TRI_ALL_VIEWS — one 2·n_cam_idx x 4 DLT over all listed views
 *              (BASELINE config 3), parameters of camera cam_idx[i].
 * out_xyz_dev  : [n_points][3] float32 (cv.convertPointsFromHomogeneous result).
 * out_xyzw_dev : optional [n_points][4] float64 null vector (may be NULL).
 * ------------------------------------------------------------------------- */
#define MVP_TRI_REFERENCE 0
#define MVP_TRI_ALL_VIEWS 1

int mvp_triangulate(const float* kpts_dev, int64_t n_points, int V, const double* cams_dev,
                    int n_cams, const int* cam_idx_host, int n_cam_idx, int mode,
                    float* out_xyz_dev, double* out_xyzw_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MVPOSE_H */
