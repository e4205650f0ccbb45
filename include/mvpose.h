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
/* OR-ed into mode: solve every point with the exact JacobiSVDImpl_ restatement
 * (default: QR + inverse iteration, Jacobi where that has not converged or its f32
 * outputs are not certified equal to Jacobi's: the same float32 bits either way). */
#define MVP_TRI_EXACT_JACOBI 0x10
/* OR-ed into mode: throughput solver whose float32 outputs are certified bit-identical to the
 * exact path's (mixed f32/fp64 undistortion, normal-equation inverse iteration; a point whose
 * f32 roundings fall inside the error bound is re-solved on the exact path by a second launch).
 * The certification is EMPIRICAL, not a proof: the null vector's rounding-floor term uses
 * constants fitted on 1.4 M synthetic and random points (the exact Jacobi's own error measured
 * <= 0.025 eps*sqrt(trM/D2) where 0.2 is used, and D2/lambda3 <= 1.4; triangulate.hip
 * null_vector_delta2).  tests/test_triangulate_gpu.py also asserts bit-identity on adversarial rigs (tiny
 * baselines, points near the epipoles, near-parallel rays).  Pass MVP_TRI_EXACT_JACOBI where a
 * proof is required.
 * Reference mode with 2 listed cameras; other cases run the default solver.  With
 * out_xyzw_dev != NULL every point takes the exact path (the float64 vectors are diagnostics). */
#define MVP_TRI_TOLERANCE 0x20

int mvp_triangulate(const float* kpts_dev, int64_t n_points, int V, const double* cams_dev,
                    int n_cams, const int* cam_idx_host, int n_cam_idx, int mode,
                    float* out_xyz_dev, double* out_xyzw_dev, void* stream);

/* Points the MVP_TRI_TOLERANCE solver re-solved on the exact path on this stream so far
 * (observability; synchronises the stream).  No reference counterpart. */
int mvp_triangulate_fallback_total(void* stream, unsigned long long* out_total_host);

/* ---------------------------------------------------------------------------
 * mvp_triangulate_points_f64 — replaces utils.triangulate_points (utils.py:1277-1336)
 * called with float64 keypoints, as the extrinsic branch does on its Gaussian samples
 * (pose_refinement.py:811): OpenCV keeps CV_64F through undistortPoints, triangulatePoints
 * and convertPointsFromHomogeneous, so nothing is rounded to f32.
 *
 * kpts_dev : [n_points][2 views][2] float64 (the reference's (n_pts, 2, 2) layout).
 * cams_dev : [2][MVP_CAM_DOUBLES] float64, camera 1 then camera 2; P (slots 26..37) as the
 *            caller computed it (the reference's np.dot in the parameters' own dtype).
 * out_xyz_dev  : [n_points][3] float64.  out_xyzw_dev: optional [n_points][4] float64.
 * Exact JacobiSVDImpl_ restatement for every point.
 * ------------------------------------------------------------------------- */
int mvp_triangulate_points_f64(const double* kpts_dev, int64_t n_points, const double* cams_dev,
                               double* out_xyz_dev, double* out_xyzw_dev, void* stream);

/* ---------------------------------------------------------------------------
 * 2D stage around the backbone (replaces, per camera frame, what
 * PoseEstimator.predict gets from mmpose at mmpose_pose_estimation.py:253-267).
 *
 * mvp_preprocess: TopdownAffine for each crop's bbox + PoseDataPreprocessor.
 *   frames_dev [n][H][W][3] uint8 (as the reference hands them to the model);
 *   minv_dev [n][6] float64 = the crop -> image map cv2.warpAffine uses
 *   internally (inverse of mmpose get_warp_matrix); mean3/std3 host f32;
 *   swap_rb = bgr_to_rgb.  out_dev [(1+with_flip)*n][out_h][out_w][4] bf16
 *   (RGB + zero channel); the flipped copies (flip test) follow the n originals.
 * mvp_heatmap_decode: flip-test average (flip_mode='heatmap', shift_heatmap)
 *   + MSRAHeatmap decode + restore to image pixels.  hm_dev/hm_flip_dev
 *   [N][K][H][W] f32 (hm_flip may be NULL: no flip test); flip_idx_host [K];
 *   center_scale_dev [N][4] f32 (cx, cy, sw, sh); outputs avg_dev (nullable)
 *   [N][K][H][W], kpts_dev [N][K][2] f32, scores_dev [N][K] f32, argmax_dev
 *   (nullable) [N][K] int32 flat index into H*W; kpts_tkv_dev (nullable)
 *   [N/V][K][3][V] f32 = the reference kpts_2d layout (crops ordered (t, v)).
 * mvp_heatmap_moments: revert_heatmap (warp of each map to the img_h x img_w
 *   image, float bilinear) fused with get_heatmap_means_cov
 *   (mmpose_pose_estimation.py:163-215): out_dev [N][K][6] float64
 *   (mx, my, vxx, vxy, vxy, vyy); minv_dev [N][6] = image -> heatmap map;
 *   separable != 0 asserts (host-checked with mvp_warp_is_separable) that every
 *   map's fixed-point source column depends on x only and source row on y only,
 *   enabling the column-resident fast path (per run of rows sharing a source
 *   row, columns whose taps are all clearly above / below thr are summed in
 *   closed form); separable == 2 runs that path walking every row of every
 *   column (diagnostics, tests).  separable_dev (nullable) [N] int: per-crop flags
 *   from mvp_bbox_geometry; crops flagged 0 take the general path, the others the
 *   `separable` mode.
 * ------------------------------------------------------------------------- */
int mvp_preprocess(const uint8_t* frames_dev, int n, int H, int W, const double* minv_dev, int out_h, int out_w,
                   const float* mean3_host, const float* std3_host, int swap_rb, int with_flip, uint16_t* out_dev,
                   void* stream);
int mvp_heatmap_decode(const float* hm_dev, const float* hm_flip_dev, int N, int K, int H, int W,
                       const int* flip_idx_host, int shift, const float* center_scale_dev, int input_w, int input_h,
                       float* avg_dev, float* kpts_dev, float* scores_dev, int32_t* argmax_dev, float* kpts_tkv_dev,
                       int V, void* stream);
int mvp_warp_is_separable(const double* minv_host, int img_h, int img_w, int* separable_out);
/* revert_heatmap only (not on the hot path, which fuses it into the moments): each crop's
 * K maps [N][K][h][w] f32 warped to the image, out [N][K][img_h][img_w] f32 — cv2.warpAffine
 * INTER_LINEAR / BORDER_CONSTANT with minv = the image -> heatmap map (as for moments). */
int mvp_heatmap_revert(const float* hm_dev, int N, int K, int h, int w, const double* minv_dev, int img_h,
                       int img_w, float* out_dev, void* stream);
int mvp_heatmap_moments(const float* hm_dev, int N, int K, int h, int w, const double* minv_dev, int img_h,
                        int img_w, float thr, int separable, const int* separable_dev, double* out_dev,
                        void* stream);
/* mvp_bbox_geometry: the reference's detector -> inference_topdown hand-off and TopdownAffine
 *   geometry on the device (replaces mmpose_pose_estimation.py:242-253 + mmpose bbox_xyxy2cs /
 *   _fix_aspect_ratio / get_warp_matrix -> cv2.getAffineTransform (cv::solve LU) and
 *   warpAffine's inversion).  Row i of boxes_dev ([n][stride] f32: x1, y1, x2, y2, ...) is the
 *   person box when its four coordinates are finite and (score_col < 0 or
 *   row[score_col] > bbox_thr), else the whole frame_w x frame_h image.  Writes crop_minv_dev
 *   [n][6] f64 (crop -> image, for mvp_preprocess), revert_minv_dev [n][6] f64 (image ->
 *   heatmap, for mvp_heatmap_moments / revert), center_scale_dev [n][4] f32 (for
 *   mvp_heatmap_decode) and separable_dev [n] int (mvp_warp_is_separable of the revert map).
 *   Fed directly with mvp_det_forward's best_dev (stride 6, score_col 4). */
int mvp_bbox_geometry(const float* boxes_dev, int stride, int n, int score_col, float bbox_thr, int frame_h,
                      int frame_w, double* crop_minv_dev, double* revert_minv_dev, float* center_scale_dev,
                      int* separable_dev, void* stream);

/* ---------------------------------------------------------------------------
 * Backbone graph runtime (replaces the HRNet-W32 forward inside mmpose's
 * inference_topdown, called at mmpose_pose_estimation.py:253 once per camera
 * frame, batch 1, on the CPU).  A static graph of convolutions on bf16 NHWC
 * activations, BN folded into the weights, executed batch-wide on one stream.
 * The graph (topology + packed weights) is built by the host
 * (mvpose/hrnet.py); the runtime validates it, plans one activation arena by
 * tensor liveness (buffers reused across the ~330 ops), and launches the HIP
 * kernels.
 *
 * Tensors: per-crop shape (h, w, c); dtype MVP_DT_BF16_NHWC or
 * MVP_DT_F32_NCHW.  The batch dimension is given at forward time.
 * Ops:
 *   MVP_OP_STEM : 3x3/s2 conv of a 4-channel (RGB+0) bf16 input to 64 ch, BN+ReLU
 *                 folded; w_off/b_off index the f32 blob ([64][3][3][4], [64]).
 *   MVP_OP_CONV : y = act(conv(in[0]) + bias [+ in[1]]), ks 1|3, stride 1|2;
 *                 w_off indexes the bf16 blob ([cout_pad][ks][ks][cin]),
 *                 b_off the f32 blob ([cout_pad]); cout_pad = cout <= 32 ? 32 :
 *                 round_up(cout, 64).  An F32_NCHW output tensor makes it the
 *                 heatmap head.
 *   MVP_OP_FUSE : out = act(sum_k nearest_upsample(in[k], up[k])), n_in <= 4
 *                 (HRModule multi-scale fuse).
 * Segments: every op carries a segment id; the ops of a segment are
 * contiguous.  seg_micro_batch_host[g] > 0 runs segment g in micro-batches of
 * that many crops (0 = whole batch at once): tensors produced and consumed only
 * inside a micro-batched segment are allocated for one micro-batch, so a chain
 * of layers keeps its intermediates in the 256 MiB Infinity Cache instead of
 * HBM.
 * ------------------------------------------------------------------------- */
#define MVP_DT_BF16_NHWC 0
#define MVP_DT_F32_NCHW 1

#define MVP_OP_STEM 0
#define MVP_OP_CONV 1
#define MVP_OP_FUSE 2

typedef struct mvp_tensor_desc {
    int h, w, c, dtype;
} mvp_tensor_desc;

typedef struct mvp_op_desc {
    int kind;
    int out;
    int n_in;
    int in[4];
    int up[4];
    int cin, cout, ks, stride, relu;
    int segment;
    int64_t w_off;
    int64_t b_off;
} mvp_op_desc;

int mvp_graph_create(const mvp_tensor_desc* tensors_host, int n_tensors, const mvp_op_desc* ops_host, int n_ops,
                     const int* seg_micro_batch_host, int n_segments, int input_tensor, int output_tensor,
                     const uint16_t* w_bf16_dev, int64_t w_elems, const float* f32_dev, int64_t f32_elems,
                     int max_batch, void** handle_out);
/* input_dev: [batch][h][w][c] of the input tensor; output_dev: the output tensor. */
int mvp_graph_forward(void* handle, const void* input_dev, int batch, void* output_dev, void* stream);
int mvp_graph_arena_bytes(void* handle, int64_t* bytes_out);
/* The weight blobs passed to mvp_graph_create were rewritten in place (e.g. an RCCL
 * broadcast from rank 0 after every rank built its graph): re-derive every weight
 * the graph copied out of them at create time (cat-fused 1x1 weights / biases, the
 * sibling-fused 3x3/s2 weights, and the slot-order weight images of the 128/256-channel
 * branch planes, the streamed-weight 3x3/s2 convs and transition1).
 * Blocking (device-synchronising). */
int mvp_graph_refresh_weights(void* handle);
int mvp_graph_destroy(void* handle);
/* Diagnostics (no reference counterpart): the kernel launches one mvp_graph_forward of `batch`
 * crops issues, in order, as records of 4 int64 {launching op, route, crops, MACs of every op
 * the launch covers}; route 1 fused BasicBlock, 2 transition twin, 3 s2 siblings, 4 head +
 * fuse, 5 Bottleneck, 6 stem pair, 7 stem, 8 conv, 9 1x1 pair, 10 fuse sum.  Fails unless every
 * op is covered by exactly one launch.  *covered_macs_out (optional) = the sum.
 * tools/fwd_breakdown.py pairs the records with a kernel trace. */
int mvp_graph_plan(void* handle, int batch, int64_t* rec_out, int max_records, int* n_records,
                   int64_t* covered_macs_out);

/* ---------------------------------------------------------------------------
 * Person detector: RTMDet-m (the reference's `detectors.coco_base`,
 * examples/model_paths.yaml:2-4) as run by PoseEstimator.predict through mmdet's
 * inference_detector (mmpose_pose_estimation.py:98-99, :234-241), followed by the
 * reference's hand-off rule (:242-250): the first detection with label 0 and score >
 * bbox_thr.  After mmdet's NMS the first detection is the highest-scoring prior that
 * survives score_thr and the min-size filter, so the hot path is: letterbox ->
 * CSPNeXt-m / CSPNeXtPAFPN / RTMDetSepBNHead -> per-prior score + box -> per-frame
 * argmax.  A per-frame NMS kernel gives mmdet's full detection list.
 *
 * mvp_det_letterbox: frames_dev [n][h][w][3] uint8 -> out_dev [n][size][size][4] bf16:
 *   mmdet Resize(scale=(size, size), keep_ratio=True) with cv2 INTER_LINEAR semantics
 *   (exact 2x downscale = INTER_AREA's fast path), Pad(114) bottom / right, then
 *   (x - mean[c]) / std[c] in f32 (channel 3 = 0).  new_h / new_w are the resized extent
 *   (mmcv rescale_size: int(h * s + 0.5), s = min(size / long, size / short)).
 *
 * Graph ops (views = channel slices of NHWC bf16 tensors: concat is a shared buffer):
 *   MVP_DET_STEM : 3x3/s2 conv of the 4-channel letterboxed input to 32 channels,
 *                  f32 weights [32][3][3][4] + bias [32], act.
 *   MVP_DET_CONV : y = act(conv(x) + bias [+ res]), ks 1|3, stride 1|2, bf16 weights
 *                  [cout_pad][ks][ks][cin] (cout_pad as mvp_graph), f32 bias.  aux = the live
 *                  couts L (0 = all): the caller guarantees zero weights and bias for couts
 *                  >= L, whose outputs are then stored as 0 without being computed.
 *   MVP_DET_DW   : 5x5 depthwise conv + bias + act, f32 weights [c/8][25][8], bias [c].
 *   MVP_DET_CA   : channel attention in place on `in`: x *= hardsigmoid(W·mean(x) + b),
 *                  f32 W^T [c][c] (w_off) and b [c].
 *   MVP_DET_SPP  : `in` = slice 0 (c channels) of a 4c buffer; writes max-pools 5/9/13
 *                  (stride 1, -inf padding) into slices 1..3.
 *   MVP_DET_UP2  : out = nearest 2x upsample of in.
 *   MVP_DET_HEAD : one FPN level's predictions from `in` = [cls feat | reg feat]
 *                  (c = 2 * 192): f32 weights [5][192] (cls, reg l/t/r/b) + bias [5];
 *                  writes cand rows [prior][6] = {sigmoid score, x1, y1, x2, y2, logit}
 *                  at prior offset `aux`, box = prior (x, y) * stride -+ exp(reg) * stride,
 *                  clipped to [0, size] (mmdet distance2bbox on img_shape).
 *   MVP_DET_DWPW : a CSPNeXtBlock's conv2 (DepthwiseSeparableConvModule) in one launch:
 *                  t = act(dw5x5(in) + b_dw) rounded to bf16 (never stored), then
 *                  out = act(t . W_pw + b_pw) [+ res]; in.c = C in {64, 96},
 *                  cout_pad(out.c) == C.  w_off: dw f32 weights [C/8][25][8]; b_off: f32
 *                  [b_dw (C) | b_pw (C)]; aux: pw bf16 weights [C][1][1][C].  Bit-identical to
 *                  MVP_DET_DW followed by a 1x1 MVP_DET_CONV.
 * act: 0 none, 1 ReLU (after a residual add), 2 SiLU (before it: CSPNeXtBlock's
 * conv2(conv1(x)) + x).
 * ------------------------------------------------------------------------- */
#define MVP_DET_STEM 0
#define MVP_DET_CONV 1
#define MVP_DET_DW 2
#define MVP_DET_CA 3
#define MVP_DET_SPP 4
#define MVP_DET_UP2 5
#define MVP_DET_HEAD 6
#define MVP_DET_DWPW 7

typedef struct mvp_det_view {
    int t;    /* tensor id, -1 = none */
    int coff; /* first channel of the slice */
    int c;    /* channels of the slice */
} mvp_det_view;

typedef struct mvp_det_op {
    int kind;
    mvp_det_view in, out, res;
    int ks, stride, act;
    int64_t w_off, b_off;
    int64_t aux;
} mvp_det_op;

int mvp_det_letterbox(const uint8_t* frames_dev, int n, int h, int w, int size, const float* mean3_host,
                      const float* std3_host, void* out_dev, void* stream);
/* tensors_host: (h, w, c, unused) per image; tensor `input_tensor` is the letterboxed image
 * (c = 4).  n_priors = total rows the HEAD ops write. */
int mvp_det_create(const mvp_tensor_desc* tensors_host, int n_tensors, const mvp_det_op* ops_host, int n_ops,
                   int input_tensor, int size, int n_priors, const uint16_t* w_bf16_dev, int64_t w_elems,
                   const float* f32_dev, int64_t f32_elems, int max_batch, void** handle_out);
/* frames_dev [n][h][w][3] uint8 -> cand_dev [n][n_priors][6] f32 and best_dev [n][6] f32 =
 * {x1, y1, x2, y2, score, prior} of the highest-scoring prior with score > score_thr and a
 * positive width / height after rescaling to the frame (x / (new_w / w), y / (new_h / h));
 * ties -> lowest prior index; score = -1 when none.  letterboxed_dev: NULL (internal) or a
 * caller buffer [n][size][size][4] bf16 that receives the letterboxed input. */
int mvp_det_forward(void* handle, const uint8_t* frames_dev, int n, int h, int w, float score_thr, float* cand_dev,
                    float* best_dev, void* letterboxed_dev, void* stream);
/* mmdet post-processing on cand_dev from mvp_det_forward: per frame, priors with score >
 * score_thr, the nms_pre best of each level (level l = prior rows [level_off[l],
 * level_off[l + 1])), boxes rescaled to the frame, min-size filter, greedy NMS at iou_thr
 * in descending score order (ties: lower prior first), the first max_det kept ->
 * dets_dev [n][max_det][5] {x1, y1, x2, y2, score} (score-descending), counts_dev [n]. */
int mvp_det_nms(const float* cand_dev, int n, int n_priors, const int* level_off_host, int n_levels, int nms_pre,
                float score_thr, float iou_thr, int max_det, float fx, float fy, float* dets_dev, int* counts_dev,
                void* stream);
int mvp_det_arena_bytes(void* handle, int64_t* bytes_out);
/* Layer-by-layer access for parity tests: mvp_det_run_ops runs the letterbox (when
 * op_begin == 0) and ops [op_begin, op_end) on the handle's arena; mvp_det_tensor_copy
 * copies the first n images of arena tensor t to (to_arena = 0) or from (1) buf_dev. */
int mvp_det_run_ops(void* handle, const uint8_t* frames_dev, int n, int h, int w, int op_begin, int op_end,
                    float* cand_dev, void* stream);
int mvp_det_tensor_copy(void* handle, int t, int n, void* buf_dev, int to_arena, void* stream);
/* Producer passes folded into their consumer 1x1 conv at create time (the neck's nearest-2x
 * upsamples; the channel-attention scale pass): folded_out[k] = 1 when op k's pass runs inside
 * the next conv reading its tensor (a DET_UP2 then launches nothing and leaves its output slice
 * unwritten; a DET_CA computes its scales and leaves its tensor unscaled); folded_out[0] = 2
 * when the letterbox runs inside the stem (op 0 stages its rows from the raw frames; the input
 * tensor stays unwritten unless mvp_det_forward is given letterboxed_dev); else 0.  Off with
 * MVPOSE_DET_FOLD=0 in the environment at create time.  Results are bit-identical either way. */
int mvp_det_folded_ops(void* handle, int* folded_out, int n_ops);
int mvp_det_destroy(void* handle);

/* ---------------------------------------------------------------------------
 * Reprojection-error trajectory refinement (Optimized_3d_Pose_Estimation,
 * reference pose_refinement.py:579-668 + sgd_optimize :894-1096, trajectory-only
 * path the CLI runs at :1210-1214).
 *
 * One workgroup refines one trajectory: the whole optimisation (every
 * iteration, every overlapping window, forward costs, analytic gradient,
 * clip_grad_norm_, Adam, running-mean early stop, best-trajectory snapshot)
 * runs inside ONE launch.  M independent trajectories run as M workgroups.
 *
 * Camera record (MVP_SGD_CAM_FLOATS f32): [K 9 | R 9 (matrix) | T 3 | dist 5].
 * ------------------------------------------------------------------------- */
#define MVP_SGD_CAM_FLOATS 26
#define MVP_SGD_N_COSTS 4 /* total, likelihood, smoothness, body_length */

typedef struct mvp_sgd_params {
    /* Python floats in the reference: kept in double so the f32 casts match torch's. */
    double lr, beta1, beta2, adam_eps;        /* torch.optim.Adam (eps 1e-8) */
    double lambda_smooth, lambda_body_length; /* a cost is skipped when its lambda <= 0 (:978-983) */
    double tolerance;                         /* running-mean improvement threshold (:1073) */
    double max_grad_norm;                     /* clip_grad_norm_ max_norm (1.0 at :1045) */
    int patience, max_iter;                  /* loop runs while no_improve < patience && it <= max_iter */
    int batch_size;                          /* window length; windows start every batch_size/2 (:786-796) */
    int ignore_distortions;
    int own_camera_gaussians;                /* 0 = reference: all cameras vs camera-0 Gaussians (:663, :885) */
} mvp_sgd_params;

/* Float workspace needed by mvp_sgd_refine for M trajectories of T x J points seen by V cameras. */
int mvp_sgd_workspace_floats(int M, int T, int V, int J, int64_t* out);

/* gauss [M][T][V][J][6] f32 (mx,my,cxx,cxy,cyx,cyy), traj0 [M][T][J][3] f32 (T already sliced by
 * time_interval; windows cover the first floor(T/batch_size)*batch_size rows), cams [V][26] f32, seg [n_seg][2] int
 * joint pairs (a -> b, length |X_b - X_a|) with seg_len [n_seg] f32 in the body-length YAML order.
 * Outputs: final [M][T][J][3], best [M][T][J][3] (NaN if never improved),
 * batch_costs [M][max_iter+1][n_windows][4], iter_means [M][max_iter+1][4] (the reference's
 * running means), iters [M] (iterations executed).  All pointers are device pointers except p. */
int mvp_sgd_refine(const float* gauss, const float* traj0, const float* cams, int M, int T, int V, int J,
                   const int* seg, const float* seg_len, int n_seg, const mvp_sgd_params* p, float* workspace,
                   float* final_traj, float* best_traj, float* batch_costs, float* iter_means, int* iters,
                   void* stream);

/* Joint trajectory + extrinsic refinement: sgd_optimize(extrinsic_optimization_IDs=ids,
 * optimize_trajectory=True) (pose_refinement.py:894-1096 with :931-954 — the listed cameras'
 * R (3x3 matrix, the reference's default learnable form) and T are leaf tensors in the same
 * Adam optimizer as the trajectory, ahead of it, and in the same clip_grad_norm_).  As
 * mvp_sgd_refine, plus learn_cam_host [n_learn] (host) camera slots (0 <= slot < V, distinct,
 * n_learn <= 2) whose R, T receive the likelihood gradient (dcost/dR_ij = dcost/dP_i X_j,
 * dcost/dT_i = dcost/dP_i, P = R X + T) and their own Adam state.  cams_final / cams_best
 * [M][n_learn][12] f32 (R row-major | T; best = NaN if never improved) are device pointers;
 * the cams records themselves are not modified. */
int mvp_sgd_refine_cams(const float* gauss, const float* traj0, const float* cams, int M, int T, int V, int J,
                        const int* seg, const float* seg_len, int n_seg, const mvp_sgd_params* p, float* workspace,
                        float* final_traj, float* best_traj, float* batch_costs, float* iter_means, int* iters,
                        const int* learn_cam_host, int n_learn, float* cams_final, float* cams_best, void* stream);

/* project_points_torch (pose_refinement.py:94-179): pts [n][3] f32 -> uv [n][2] f32 for one camera
 * record (R as a 3x3 matrix). */
/* Extrinsic-from-samples refinement (sgd_optimize(extrinsic_optimization_IDs=[id],
 * optimize_trajectory=False), reference pose_refinement.py:684-706, :800-831, :915-943):
 * one pass over the triangulated Gaussian samples samples_dev [n_points][3] f32, ordered
 * (t, joint, sample) with n_samples per (t, joint); targets_dev [n_points / n_samples][6] f32
 * = (mean x, mean y, Σ⁻¹ 00, 01, 10, 11) per (t, joint); cam_dev = the learnable camera's
 * MVP_SGD_CAM_FLOATS record (R as a matrix).  Writes per-block fp64 partial sums
 * partial_dev [n_blocks][14] = [Σ 0.5 dᵀΣ⁻¹d over finite terms, finite count, Σ dq/dR (9,
 * row-major), Σ dq/dT (3)]; the caller reduces them (cost = sum / count, gradients / count). */
int mvp_extrinsic_sample_grad(const float* samples_dev, const float* targets_dev, int n_samples, int64_t n_points,
                              const float* cam_dev, int ignore_distortions, int n_blocks, double* partial_dev,
                              void* stream);
/* One Adam step of that branch on the device (pose_refinement.py:1039-1050, learnable R as a
 * 3x3 matrix and T): reduces partial_dev [n_blocks][14] of mvp_extrinsic_sample_grad, casts
 * cost and gradient to f32 like the host path, clip_grad_norm_([R, T], max_norm), torch
 * single-tensor Adam on R and T with state_dev [m (12) | v (12) | step (int32)] (zero it before
 * the first step), and updates R (cam_dev[9..18)) and T (cam_dev[18..21)) in place, so the next
 * mvp_extrinsic_sample_grad sees the new camera.  The step's cost goes to cost_hist_dev[step-1]
 * and the new R, T (12 floats) to param_hist_dev[step-1][12]: the host reads the history every
 * few iterations for the early-stop bookkeeping instead of once per step. */
int mvp_extrinsic_adam_step(const double* partial_dev, int n_blocks, float* cam_dev, float* state_dev, double lr,
                            double beta1, double beta2, double adam_eps, double max_norm, float* cost_hist_dev,
                            float* param_hist_dev, void* stream);
int mvp_project_points(const float* pts, int64_t n, const float* cam, int ignore_distortions, float* uv,
                       void* stream);

/* ---------------------------------------------------------------------------
 * linear_interpolation (pose_refinement.py:15-84; always run by the refinement
 * CLI, :1170-1172): outlier-filtered local linear fit per (t, point, dim).
 * pts_dev/out_dev [T][P][D] f32; k <= 30; see csrc/interp.hip for the rules.
 * ------------------------------------------------------------------------- */
int mvp_linear_interpolation(const float* pts_dev, int T, int P, int D, int k, float k_std, float median_std,
                             int use_rolling_average, int filter_distance_from_median, float* out_dev,
                             void* stream);

/* ---------------------------------------------------------------------------
 * MPEG-4 Part 2 ('mp4v') decoding, host side — replaces cv.VideoCapture on the reference's
 * recordings (utils.py:849-909 read_video_as_frames; synchronize_videos.py:64,240 writes them with
 * cv2.VideoWriter_fourcc(*'mp4v')).  Simple Profile: I / P-VOPs, video packets, H.263 or MPEG
 * quantisation; frames out as BGR24 (cv2's channel order) or I420.  No device memory involved.
 *
 * mvp_mp4v_create : config = the VOS/VO/VOL headers (an MP4 'esds' DecoderSpecificInfo, or the
 *                   head of an elementary stream); returns the frame size.
 * mvp_mp4v_decode : one sample (any GOV / VOL headers and VOPs it holds); writes the frame after
 *                   its last VOP (a not-coded VOP repeats the previous frame) to bgr_out
 *                   [H][W][3] and / or yuv_out (I420, W x H luma then two (W+1)/2 x (H+1)/2
 *                   chroma planes); *vops_out = VOPs in the sample.
 * mvp_mp4v_selfcheck : verifies the decoder's VLC / scan tables (prefix-free, complete, the intra
 *                   TCOEF codes a permutation of the inter ones, LMAX order).
 * ------------------------------------------------------------------------- */
int mvp_mp4v_create(const uint8_t* config, size_t config_bytes, void** handle, int* width, int* height);
int mvp_mp4v_decode(void* handle, const uint8_t* data, size_t bytes, uint8_t* bgr_out, uint8_t* yuv_out,
                    int* vops_out);
int mvp_mp4v_destroy(void* handle);
int mvp_mp4v_selfcheck(void);

/* Split decode: the host entropy-decodes, the device reconstructs (bit-identical to
 * mvp_mp4v_decode's frames; the decoded frames land in device memory).
 *
 * mvp_mp4v_parse : one sample with at most one VOP, on a handle that never decodes.  Writes one
 *                  32-byte record per macroblock, raster order, to rec_out (host memory, rec_cap
 *                  records >= macroblocks):
 *                    uint8 kind (0 intra, 1 inter, 2 not coded = copy, 3 not reached), uint8 nnz[6],
 *                    uint8 pad, int16 mv[4][2] (luma 8x8 vectors, half-pel), int16 cmv[2] (chroma),
 *                    uint32 first coefficient entry;
 *                  and the inverse-quantised coefficients as uint32 entries (raster position << 16 |
 *                  uint16 value), block by block, to coef_out (*n_coef entries, at most coef_cap;
 *                  384 per macroblock always suffices).  vop_out[0] = 1 coded VOP, 0 not coded,
 *                  -1 no VOP in the sample; vop_out[1] = vop_rounding_type.
 * mvp_mp4v_reconstruct : stream-ordered; jobs_dev = n_jobs device records of 48 bytes
 *                  {const rec*, const coef*, uint8 cur*, const uint8 ref*, uint8 bgr* or NULL,
 *                   int32 coded, int32 rounding}, all device pointers: the VOP's records and
 *                  entries, the picture it writes and the previous one (each an I420 picture with
 *                  macroblock-aligned planes: Y 16*mb_w x 16*mb_h, then U and V 8*mb_w x 8*mb_h;
 *                  a slot's first pictures hold 128), and the [height][width][3] BGR frame out.
 *                  Jobs must write distinct pictures; a coded VOP's cur is the slot's older
 *                  picture (the host decoder's swap), a not-coded VOP outputs cur unchanged. */
int mvp_mp4v_parse(void* handle, const uint8_t* data, size_t bytes, void* rec_out, int64_t rec_cap,
                   uint32_t* coef_out, int64_t coef_cap, int64_t* n_coef, int* vop_out);
int mvp_mp4v_reconstruct(const void* jobs_dev, int n_jobs, int width, int height, void* stream);
/* mvp_mp4v_parse over samples data[0..n) in one call (one GIL release per GOP from Python):
 * sample k's records at rec_out + k * 32 * macroblocks, its coefficients packed after sample
 * k-1's in coef_out (n_coef[k] entries), vop_out[2k..2k+1].  Stops before a sample that might not
 * fit (fewer than 384 entries per macroblock left); *n_done = samples parsed. */
int mvp_mp4v_parse_many(void* handle, int n, const uint8_t* const* data, const size_t* bytes, void* rec_out,
                        uint32_t* coef_out, int64_t coef_cap, int64_t* n_coef, int* vop_out, int* n_done);

#ifdef __cplusplus
}
#endif
#endif /* MVPOSE_H */
