"""Benchmark: multi-view frames/s end to end (2-cam HRNet-W32 256x192 bf16, 17 kpts).

One step = one pass of the hot path over one batch of synthetic input already
resident in HBM: B synchronised frames x V cameras (uint8 1280x720) ->
crop + normalise -> HRNet-W32 with flip test (2·B·V crops, bf16 MFMA) ->
flip-average + MSRA decode -> revert + heatmap moments -> batched DLT
triangulation (BASELINE.json configs[1]).  Multi-GPU (torchrun): frames are
sharded across ranks (weak scaling); weights are broadcast once over RCCL and
each step's 3D joints are gathered to rank 0 (the only collectives).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B] [--views V]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA spec
METRIC = "multi-view frames/sec end-to-end (2-cam HRNet-W32, 17 kpts) at 1/2/4/8 GPUs"
TRI_T = 1_000_000           # frames per triangulation-roofline launch: 612 MB (V=2) / 1.02 GB (V=4)
                            # per launch, well past the 256 MiB Infinity Cache -> an HBM measurement
SGD_V, SGD_T, SGD_M = 8, 400, 256   # BASELINE config 5 (V=8, T=400); M trajectories per launch
SGD_ITERS = 40
SGD_BENCH_ATOL = 2e-4      # cm, final trajectory vs the reference after 40 Adam iterations
# FP32 FLOP per (frame, camera, joint) projection + likelihood forward + adjoint in sgd_kernel
# (csrc/sgd.hip project / quad_cost / project_adjoint, distortion on, counted by hand: DESIGN.md
# §4) and per trajectory coordinate (stencil + segment adjoints + Adam)
SGD_FLOP_PER_PROJ = 175
SGD_FLOP_PER_COORD = 25
FP32_PEAK_TFLOPS = 157.3    # vector FP32 (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=256, help="synchronised frames per step per GPU")
    ap.add_argument("--views", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frames", type=int, default=12,
                    help="frames of the all-threads CPU baseline sample (config 1 is 50 frames)")
    ap.add_argument("--cpu-sample-frames-1t", type=int, default=2, help="frames of the 1-thread sample")
    ap.add_argument("--no-extra", action="store_true", help="skip the config 3 / config 5 side lines")
    return ap.parse_args()


def spawn_ranks(n):
    """`bench.py --gpus N` without a torchrun environment: start N ranks (one process per GPU)
    through torch.distributed.run as a CHILD process, before this process touches the GPU,
    and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# The committed PMC traffic pass the roofline lines cite (tools/pmc_traffic.py): named explicitly —
# a newest-file rule picked r04zz_ over r04zz2_ by lexicographic order in round 4.
TRAFFIC_FILE = "profiles/r06u_traffic.json"
# per-kernel-family breakdown of one 1,024-crop forward (tools/fwd_breakdown.sh: a kernel trace of
# backbone forwards only, paired with the graph's launch plan for each launch's MACs)
BREAKDOWN_FILE = "profiles/r06a_forward_breakdown.json"


def committed_traffic():
    """HBM bytes per launch from the committed PMC pass TRAFFIC_FILE (2*FETCH_SIZE + WRITE_SIZE,
    gfx950-corrected) — PMC counters cannot be read from inside a normal run."""
    path = os.path.join(ROOT, TRAFFIC_FILE)
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        return json.load(f), TRAFFIC_FILE


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", local if world > 1 else 0)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_path(n_frames, views, seed=0):
    """The reference-equivalent CPU path (oracle restatement):
    torch-CPU fp32 HRNet-W32 at batch 1 per camera with flip test, numpy decode,
    revert + moments, OpenCV-semantics triangulation.  Returns seconds."""
    sys.path.insert(0, ROOT)
    from oracle import cv_ref, heatmap_ref, hrnet_ref
    from mvpose import hrnet, synthetic as syn
    model = hrnet_ref.build(hrnet.random_state_dict(seed))
    cams = syn.make_rig(views, seed=1)
    cp = syn.reference_camera_params(cams)
    frames = syn.make_frames(n_frames * views, seed=2).reshape(n_frames, views, 720, 1280, 3)
    M, center, scale = heatmap_ref.topdown_crop_matrix(1280, 720)
    Mh = heatmap_ref.get_warp_matrix(center, scale, 0.0, (48, 64), inv=True)
    t0 = time.perf_counter()
    kpts = np.zeros((n_frames, 17, 3, views), np.float32)
    for t in range(n_frames):
        for v in range(views):
            x = torch.from_numpy(heatmap_ref.preprocess(frames[t, v], M))[None]
            avg, _, _ = hrnet_ref.flip_test_forward(model, x)
            k, sc, _ = heatmap_ref.msra_decode(avg[0].numpy())
            kpts[t, :, :2, v] = heatmap_ref.keypoints_to_image(k, center, scale)
            kpts[t, :, 2, v] = sc
            heatmap_ref.heatmap_means_cov_f64(heatmap_ref.warp_affine_linear_f32(avg[0].numpy(), Mh, 720, 1280))
    cv_ref.get_pose_3D(cp, kpts, camera_indices=[0, 1])
    return time.perf_counter() - t0


def cpu_baseline(n_frames, n_frames_1t, views):
    """Config 1 on this host's cores: all threads, then 1 thread, each on a
    bounded sample of the 50-frame config so the default bench stays within minutes."""
    n_threads = torch.get_num_threads()
    dt = _cpu_path(n_frames, views)
    torch.set_num_threads(1)
    try:
        dt1 = _cpu_path(n_frames_1t, views) if n_frames_1t > 0 else None
    finally:
        torch.set_num_threads(n_threads)
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    out = {"value": n_frames / dt, "unit": "frames/s", "cores": n_threads, "kind": "port",
           "host_cpu_count": os.cpu_count(), "usable_cpus": usable, "cpu_model": _cpu_model(),
           "threads_note": "cores = torch.get_num_threads() = the intra-op threads the sample ran on; torch takes "
                           "it from OMP_NUM_THREADS, which the GPU box sets to its per-GPU CPU share (16); "
                           "usable_cpus = this process's affinity mask (the box's whole machine is shared)",
           "sample": f"{n_frames} of config 1's 50 synthetic {views}-cam 1280x720 frames, batch 1 per camera, "
                     f"flip test, {dt:.1f} s on {n_threads} threads (oracle/ restatement: torch-CPU fp32 "
                     f"HRNet-W32 + numpy decode/revert/moments + OpenCV-4.9-semantics triangulation in C)"}
    if dt1 is not None:
        out["value_1thread"] = n_frames_1t / dt1
        out["sample_1thread"] = f"{n_frames_1t} frames, {dt1:.1f} s on 1 thread"
    return out


# Triangulation's real bound is VALU issue (fp64 undistortion + solver), read from a committed PMC
# pass of the same kernel (tools/tri_pmc_json.py): valu_busy = SQ_ACTIVE_INST_VALU x 4 cycles per
# SIMD over GRBM_GUI_ACTIVE / 8 cycles per XCD, at the clock the chip held in that pass
# (GRBM_GUI_ACTIVE / 8 / dispatch duration).  The issue floor at that clock is the busy cycles'
# share of the launch: floor_ms = valu_busy x the pass's duration.
TRI_TOL_PMC = "r05_tri_tol_pmc.json"
TRI_REF_PMC = "r05_tri_ref_pmc.json"


def tri_valu_issue(tri_ms, pmc_file):
    path = os.path.join(ROOT, "profiles", pmc_file)
    if not os.path.exists(path):
        return None
    pmc = json.load(open(path))
    if "valu_busy" not in pmc:
        return None
    w = pmc.get("per_wave", {})
    f64 = sum(w.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64"))
    return {"frac": pmc["valu_busy"], "clock_GHz": pmc.get("clock_GHz_median"),
            "pmc_launch_ms": pmc.get("duration_ms_median"), "bench_launch_ms": tri_ms,
            "valu_instr_per_wave": w.get("SQ_INSTS_VALU"), "f64_instr_per_wave": f64,
            "trans_f64_per_wave": w.get("SQ_INSTS_VALU_TRANS_F64"),
            "model": "frac = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8): the SIMDs' VALU-issue "
                     "share of the kernel's cycles, at the clock GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md "
                     "DVFS give-back)", "source": f"profiles/{pmc_file}"}


def tri_line(ops, syn, dev, s, views, mode, reps=10, tolerance=False):
    """One triangulation launch over a resident TRI_T-frame stream (the per-step 256-frame
    launch is latency-bound and says nothing about the kernel).  HIP events on the launch
    stream; the stream is ~2.4-4x the Infinity Cache, so every launch streams from HBM.
    tolerance=True: the throughput solver (MVP_TRI_TOLERANCE, <= 1e-4 world units against
    the exact-rounding path; its fallback launch is inside the timed region)."""
    cams = syn.make_rig(views, seed=1)
    cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device=dev)
    k = torch.tensor(syn.make_kpts_2d(syn.make_poses(2000, seed=2), cams, seed=3), device=dev)
    k = k.repeat((TRI_T + k.shape[0] - 1) // k.shape[0], 1, 1, 1)[:TRI_T].contiguous()
    ci = list(range(views)) if mode == ops.TRI_ALL_VIEWS else [0, 1]
    out = torch.empty((TRI_T, 17, 3), dtype=torch.float32, device=dev)
    for _ in range(2):
        ops.triangulate(k, cd, ci, mode=mode, out=out, tolerance=tolerance)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        ops.triangulate(k, cd, ci, mode=mode, out=out, tolerance=tolerance)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    v_used = views if mode == ops.TRI_ALL_VIEWS else 2
    nbytes = 12.0 * 17 * (v_used + 1) * TRI_T   # read x,y,conf per used view + write xyz, per joint
    gbs = nbytes / (ms * 1e-3) / 1e9
    del k, out
    return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "bytes_per_frame": 12 * 17 * (v_used + 1), "bytes_per_launch": nbytes,
            "frames_per_s": TRI_T / (ms * 1e-3), "avg_launch_ms": ms, "launches": reps,
            "workload": f"{TRI_T} resident synchronised {views}-cam frames per launch"}


def sgd_line(dev):
    """BASELINE config 5: V=8, T=400 reprojection + smoothness + body-length refinement
    (pose_refinement.py:894-1096), SGD_M trajectories per launch (one workgroup each), a fixed
    SGD_ITERS iterations (early stop disabled).  Outside the timed region of the headline."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from mvpose import refine
    from sgd_problem import BENCH_C5_ITERS, BENCH_C5_KW, bench_c5_inputs, inputs_digest
    cams, g, x0 = bench_c5_inputs(SGD_V, SGD_T)
    ref = np.load(os.path.join(ROOT, "tests", "golden", "bench_sgd_c5.npz"))
    assert str(ref["digest"]) == inputs_digest(cams, g, x0), "bench SGD problem drifted from its golden"
    assert BENCH_C5_ITERS == SGD_ITERS
    with open(os.path.join(ROOT, "tests", "golden", "body_part_lengths.json")) as f:
        lengths = json.load(f)["my_lengths"]
    camlist = [[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
    kw = dict(BENCH_C5_KW, body_lengths=dict(lengths), device=dev)
    res = {}
    for M in (1, SGD_M):
        G = torch.tensor(np.broadcast_to(g, (M,) + g.shape).copy(), device=dev)
        X = torch.tensor(np.broadcast_to(x0, (M,) + x0.shape).copy(), device=dev)
        refine.refine_trajectories(G, X, camlist, **kw)
        s = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = refine.refine_trajectories(G, X, camlist, **kw)
        e1.record(s)
        torch.cuda.synchronize()
        assert int(r["iters"].min()) == SGD_ITERS, r["iters"]
        # parity against the reference's own run of this problem (tests/golden/bench_sgd_c5.npz,
        # pose_refinement.sgd_optimize): every trajectory of the launch within SGD_BENCH_ATOL cm
        dev_max = float((r["final"] - torch.tensor(ref["final"], device=dev)).abs().max())
        assert dev_max <= SGD_BENCH_ATOL, (M, dev_max)
        res[M] = e0.elapsed_time(e1) / SGD_ITERS
        res[f"dev{M}"] = dev_max
    flop_iter = SGD_T * 17 * (SGD_V * SGD_FLOP_PER_PROJ + 3 * SGD_FLOP_PER_COORD)
    tf = flop_iter * SGD_M / (res[SGD_M] * 1e-3) / 1e12
    return {"workload": f"BASELINE config 5: V={SGD_V}, T={SGD_T}, one window, {SGD_ITERS} Adam iterations, "
                        f"lr 0.01, lambda_s 1e-6, lambda_b 1 (early stop off)",
            "parity": {"max_abs_cm_vs_reference": max(res["dev1"], res[f"dev{SGD_M}"]), "atol_cm": SGD_BENCH_ATOL,
                       "reference": "tests/golden/bench_sgd_c5.npz (pose_refinement.sgd_optimize, same problem)"},
            "ms_per_iter_1traj": res[1], "ms_per_iter_M": res[SGD_M], "M": SGD_M,
            "trajectory_iterations_per_s": SGD_M / (res[SGD_M] * 1e-3),
            "roofline": {"bound": "fp32 valu", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": tf / FP32_PEAK_TFLOPS, "flop_per_iter_per_traj": flop_iter,
                         "flop_model": f"{SGD_FLOP_PER_PROJ} FLOP per (t, v, j) projection + likelihood + "
                                       f"adjoint, {SGD_FLOP_PER_COORD} per coordinate (stencil, segments, Adam)"}}


def extrinsic_line(dev, T=1000, N=100, reps=20):
    """one mvp_extrinsic_sample_grad pass (the per-Adam-step cost + R/T gradient
    of sgd_optimize(extrinsic_optimization_IDs=[id], optimize_trajectory=False), reference
    pose_refinement.py:800-831) over T x 17 x N triangulated samples, HBM roofline on the
    12 B/sample read; plus the whole optimisation step with Adam on the device."""
    from mvpose import refine, synthetic as syn
    cams = syn.make_rig(3, seed=9)
    poses = syn.make_poses(T, seed=10)
    rng = np.random.default_rng(11)
    s3 = torch.tensor(poses[:, :, None, :] + rng.normal(0, 2.0, (T, 17, N, 3)), dtype=torch.float32,
                      device=dev).contiguous()
    uv = syn.project(poses, cams[2])
    tg = np.concatenate([uv, np.full((T, 17, 1), 1 / 9.0), np.zeros((T, 17, 2)), np.full((T, 17, 1), 1 / 9.0)], -1)
    tg = torch.tensor(tg, dtype=torch.float32, device=dev).contiguous()
    cam = torch.from_numpy(refine.camera_record(cams[2]["K"], cams[2]["R"], cams[2]["T"], cams[2]["dist"])).to(dev)
    refine.extrinsic_sample_grad(s3, tg, cam, N)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        refine.extrinsic_sample_grad(s3, tg, cam, N)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # the whole optimisation step as Optimized_3d_Pose_Estimation runs it: the gradient pass +
    # mvp_extrinsic_adam_step (clip + Adam on the device, camera record updated in place), no
    # host round trip; host_step_ms = the host's launch cost per step, step_ms = wall per step
    from mvpose._lib import call as _call
    import ctypes as _ct
    n_pts = T * 17 * N
    nb = max(1, min(1024, (n_pts + 255) // 256))
    part = torch.empty((nb, refine.EXT_SUMS), dtype=torch.float64, device=dev)
    state = torch.zeros(25, dtype=torch.float32, device=dev)
    hist = torch.zeros(reps + 3, dtype=torch.float32, device=dev)
    phist = torch.zeros((reps + 3, 12), dtype=torch.float32, device=dev)
    sp = _ct.c_void_p(s.cuda_stream)

    def _p(t):
        return _ct.c_void_p(t.data_ptr())

    def step():
        _call("mvp_extrinsic_sample_grad", _p(s3), _p(tg), N, n_pts, _p(cam), 0, nb, _p(part), sp)
        _call("mvp_extrinsic_adam_step", _p(part), nb, _p(cam), _p(state), 0.01, 0.9, 0.999, 1e-8, 1.0, _p(hist),
              _p(phist), sp)
    for _ in range(3):
        step()
    state.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    step_ms = (t1 - t0) * 1e3 / reps
    wall_ms = (t2 - t0) * 1e3 / reps
    n = T * 17 * N
    gbs = n * 12 / (ms * 1e-3) / 1e9
    return {"workload": f"T={T}, 17 joints, N={N} samples per (t, joint): {n} samples",
            "kernel": "extrinsic_grad_kernel", "avg_launch_ms": ms, "samples_per_s": n / (ms * 1e-3),
            "host_step_ms": step_ms, "step_ms": wall_ms,
            "step": "gradient pass + mvp_extrinsic_adam_step on the device (no per-step read-back)",
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "bytes_model": "12 B per sample (xyz f32); the 24 B "
                                                                    "target per (t, joint) is L2-resident"}}


def stage_lines(est, frames, traffic, reps=10):
    """SURVEY §8(d) lines for the step's small kernels at the headline batch (B·V camera-frames),
    each launch timed alone with HIP events on the launch stream: preprocess (crop +
    normalise, original + flipped), decode (flip average + MSRA), moments (revert + means /
    covariances).  Bytes per launch from the committed PMC pass (2·FETCH_SIZE + WRITE_SIZE,
    tools/pmc_traffic.py) next to the algorithmic bytes of each kernel's model."""
    import ctypes
    from mvpose._lib import call
    from mvpose.estimator import COCO_FLIP_INDICES, HEATMAP_THR, MEAN, STD
    from mvpose.hrnet import HEATMAP_HW, INPUT_HW, N_JOINTS
    dev = est.device
    n = frames.shape[0]
    h, w = frames.shape[1:3]
    s = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    p = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
    mean, std = (ctypes.c_float * 3)(*MEAN), (ctypes.c_float * 3)(*STD)
    flip = (ctypes.c_int * N_JOINTS)(*COCO_FLIP_INDICES)
    crops, hm = est.crops[: 2 * n], est.heatmaps[: 2 * n]
    avg = torch.empty((n, N_JOINTS) + HEATMAP_HW, dtype=torch.float32, device=dev)
    kp = torch.empty((n, N_JOINTS, 2), dtype=torch.float32, device=dev)
    sc = torch.empty((n, N_JOINTS), dtype=torch.float32, device=dev)
    gauss = torch.empty((n, N_JOINTS, 6), dtype=torch.float64, device=dev)
    launches = {
        "preprocess": lambda: call("mvp_preprocess", p(frames), n, h, w, p(est.crop_minv), INPUT_HW[0], INPUT_HW[1],
                                   mean, std, int(est.swap_rb), 1, p(crops), sp),
        "decode": lambda: call("mvp_heatmap_decode", p(hm[:n]), p(hm[n:]), n, N_JOINTS, HEATMAP_HW[0], HEATMAP_HW[1],
                               flip, 1, p(est.center_scale), INPUT_HW[1], INPUT_HW[0], p(avg), p(kp), p(sc), None,
                               None, 1, sp),
        "moments": lambda: call("mvp_heatmap_moments", p(avg), n, N_JOINTS, HEATMAP_HW[0], HEATMAP_HW[1],
                                p(est.revert_minv), h, w, ctypes.c_float(HEATMAP_THR), int(est.separable), None,
                                p(gauss), sp),
    }
    hm_b = N_JOINTS * HEATMAP_HW[0] * HEATMAP_HW[1] * 4          # one f32 heatmap stack per crop
    crop_b = INPUT_HW[0] * INPUT_HW[1] * 4 * 2                   # one bf16 crop (RGB + pad)
    algo = {  # algorithmic bytes per camera-frame
        "preprocess": (2 * crop_b, "writes the original + flipped bf16 crops (786 KB); reads the frame rows the "
                                   "whole-image warp touches (PMC: ~0.68 MB per camera-frame)"),
        "decode": (3 * hm_b, "reads both f32 heatmap stacks (2 x 209 KB), writes the flip average (209 KB)"),
        "moments": (hm_b, "reads the flip-averaged f32 maps (209 KB); the reverted 17x720x1280 map is never formed"),
    }
    out = {}
    for name, fn in launches.items():
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        pmc = traffic.get(name, {}).get("hbm_bytes_per_launch")
        per_unit, model = algo[name]
        gbs = per_unit * n / (ms * 1e-3) / 1e9
        line = {"kernel": {"preprocess": "preprocess_kernel", "decode": "decode_kernel",
                           "moments": "moments_kernel"}[name],
                "camera_frames_per_launch": n, "avg_launch_ms": ms, "launches": reps,
                "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": gbs / HBM_PEAK_GBS, "bytes_per_camera_frame": per_unit, "bytes_model": model,
                             "traffic": pmc}}
        if pmc:
            line["roofline"]["traffic_GBps"] = pmc / (ms * 1e-3) / 1e9
        if name == "moments":
            flop = 20.0 * N_JOINTS * h * w * n   # ~20 FLOP per (pixel, joint) of the reverted map
            line["flop_model_TFLOPs"] = flop / (ms * 1e-3) / 1e12
            line["flop_note"] = ("the per-pixel FLOP model of §8(d) (0.31 GFLOP per camera-frame) over the launch "
                                 "time; above the FP32 peak because the separable fast path sums whole column "
                                 "runs in closed form instead of walking the reverted map")
        out[name] = line
    return out


def ingest_line(est, V, n_frames=512, batch=128):
    """SURVEY §7 "host frame supply": the same 2D stage fed from HOST memory (decoded
    frames in RAM, as the reference holds whole videos, utils.py:849-909) through the
    overlapped pinned-staging / copy-stream pipeline (FrameStreamer).  PCIe-inclusive;
    never the headline value (frames resident in HBM)."""
    from mvpose.pose_estimation import FrameStreamer
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, (16, 720, 1280, 3), dtype=np.uint8)
    stacks = [np.ascontiguousarray(np.tile(base, (n_frames // 16, 1, 1, 1))) for _ in range(V)]
    fs = FrameStreamer(est, V, (720, 1280), batch)
    fs.run([s[:batch] for s in stacks])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kp, _ = fs.run(stacks)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gb = n_frames * V * 720 * 1280 * 3 / 1e9
    return {"frames_per_s": n_frames / dt, "frames": n_frames, "batch_frames": batch, "host_to_device_GBps": gb / dt,
            "path": "host RAM -> pinned staging (gather thread) -> H2D on a copy stream -> crop/HRNet/decode/"
                    "moments on the compute stream (2D stage only, serial moments)"}


def video_decode_line(gops=48, gop=12, threads=16):
    """the native MPEG-4 Part 2 decoder on a synthetic 1280x720 mp4v
    stream (GOPs of one I-VOP + 11 P-VOPs written by tests/mp4v_writer.py: ~5 % non-zero
    intra coefficients, +-3 px motion, ~1 % non-zero residuals), decoded to BGR frames in host
    RAM as cv2.VideoCapture would (utils.py:849-909): one thread, and the GOPs on a thread pool.
    Host CPU work, outside every GPU figure."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mp4v_writer as W
    from mvpose import video
    w, h = 1280, 720
    rng = np.random.default_rng(7)
    mw, mh = w // 16, h // 16

    def intra_mb():
        b = np.zeros((6, 64), np.int64)
        for n in range(6):
            b[n, 0] = rng.integers(40, 160) if n < 4 else rng.integers(80, 140)
            m = rng.random(63) < 0.05
            b[n, 1:][m] = rng.integers(-4, 5, m.sum())
        return {"q": 6, "blocks": b, "ac_pred": False}

    def inter_mb():
        b = np.zeros((6, 64), np.int64)
        m = rng.random((6, 64)) < 0.01
        b[m] = rng.integers(-2, 3, m.sum())
        return {"type": "inter", "mv": (int(rng.integers(-3, 4)), int(rng.integers(-3, 4))), "blocks": b}

    vw = W.VopWriter(w, h)
    i_vop = vw.i_vop([[intra_mb() for _ in range(mw)] for _ in range(mh)], 6)
    p_vops = [vw.p_vop([[inter_mb() for _ in range(mw)] for _ in range(mh)], 6, rounding=k % 2) for k in range(3)]
    samples = ([i_vop] + [p_vops[k % 3] for k in range(gop - 1)]) * gops
    cfg = W.vol_header(w, h)
    res = {}
    for th in (1, threads):
        video.decode_mp4v(cfg, samples[:gop], threads=th)
        t0 = time.perf_counter()
        out = video.decode_mp4v(cfg, samples, threads=th)
        res[th] = len(samples) / (time.perf_counter() - t0)
        assert out.shape == (len(samples), h, w, 3)
    host_frames = out
    # split decode: host entropy decoding on the thread pool, reconstruction on the GPU; timed
    # to the frames resident in HBM (torch.cuda.synchronize), the host frames never leave RAM
    import torch
    video.decode_mp4v_device(cfg, samples[:gop], threads=threads)
    torch.cuda.synchronize()
    best, phases = None, {}
    for _ in range(3):
        ph = {}
        t0 = time.perf_counter()
        dev_out = video.decode_mp4v_device(cfg, samples, threads=threads, timings=ph)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if best is None or dt < best:
            best, phases = dt, ph
    same = bool(torch.equal(dev_out.cpu(), torch.from_numpy(host_frames)))
    return {"frames_per_s": res[threads], "threads": threads, "frames_per_s_1thread": res[1],
            "frames": len(samples), "stream": f"1280x720 mp4v, GOP {gop} (I + {gop - 1} P), "
                                            f"{sum(map(len, samples)) * 8 / len(samples) * 30 / 1e6:.1f} Mbit/s at 30 fps",
            "path": "mvpose.video.decode_mp4v: native Simple Profile decoder (csrc/mp4v.cpp), GOPs on a thread pool",
            "device_split_decode": {
                "frames_per_s": len(samples) / best, "threads": threads, "bit_identical_to_host": same,
                "host_phases_ms": {k: (1e3 * v if isinstance(v, float) else v) for k, v in phases.items()},
                "path": "mvpose.video.decode_mp4v_device: host entropy decoding (mvp_mp4v_parse_many, one call per "
                        "GOP) on the thread pool, each GOP's records + coefficients to the device on a copy stream as "
                        "it is parsed, reconstruction (IDCT, half-pel MC, BGR) by mvp_mp4v_reconstruct on the GPU, one "
                        "launch per GOP position; frames end in HBM"}}


def detector_line(dev, est, cams_params, V, batch=None, reps=5):
    """the person detector the reference runs on every camera-frame
    (RTMDet-m, mmpose_pose_estimation.py:234-250), alone (letterbox -> graph -> per-frame
    selection, HIP events on the launch stream) and in front of the 2D->3D pipeline
    (the headline's est.max_frames camera-frames per process(): detect in max_batch chunks ->
    boxes -> crops -> HRNet -> decode -> moments -> DLT).  77.9 GFLOP per 640x640
    camera-frame (38.94 GMAC)."""
    from mvpose.pipeline import MultiViewPipeline
    from mvpose.rtmdet import RTMDetector
    # one detector forward per process() call: the whole step's camera-frames (512; 9.4 GiB of
    # activation arena).  tools/det_bench.py: 4,980 camera-frames/s at 128 per forward, 5,160 at
    # 256, 5,220 at 512 — the last round of workgroups of each conv fills more of the GPU
    batch = batch or est.max_frames
    det = RTMDetector(seed=0, max_batch=batch, device=dev)
    g = torch.Generator(device=dev).manual_seed(99)
    fr = torch.randint(0, 256, (batch, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)
    for _ in range(2):
        det.detect(fr)
    s = torch.cuda.current_stream(dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(s)
    for _ in range(reps):
        det.detect(fr)
    e[1].record(s)
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / reps
    flops = 2.0 * det.macs_per_frame * batch
    tf = flops / (ms * 1e-3) / 1e12
    pipe = MultiViewPipeline(cams_params, estimator=est, device=dev, detector=det)
    # the pipeline at the headline batch (est.max_frames camera-frames: 256 2-cam frames, the
    # detector in max_batch chunks)
    n_pipe = est.max_frames
    fr_p = fr.repeat((n_pipe + batch - 1) // batch, 1, 1, 1)[:n_pipe]
    fr2 = fr_p.reshape(n_pipe // V, V, 720, 1280, 3)
    out = {}
    for _ in range(2):
        pipe.process(fr2, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        pipe.process(fr2, out)
    torch.cuda.synchronize()
    e2e = (n_pipe // V) * reps / (time.perf_counter() - t0)
    found = float((det.best[:batch, 4] > 0.3).float().mean())
    res = {"model": "RTMDet-m 640x640 (CSPNeXt-m / CSPNeXtPAFPN / RTMDetSepBNHead, 1 class), seeded weights with "
                    "calibrated BN statistics", "batch_camera_frames": batch, "avg_launch_ms": ms,
           "camera_frames_per_s": batch / (ms * 1e-3), "frames_with_person_box": found,
           "pipeline_with_detector_frames_per_s": e2e, "pipeline_frames_per_process": n_pipe // V,
           "roofline": {"bound": "mfma", "achieved": tf, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": tf / BF16_PEAK_TFLOPS, "flops_per_launch": flops}}
    det.close()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, dev = setup_dist(args)
    from mvpose import dist as mdist, hrnet, ops, synthetic as syn
    from mvpose.estimator import BatchPoseEstimator
    from mvpose.pipeline import MultiViewPipeline

    B, V = args.frames, args.views
    est = BatchPoseEstimator(hrnet.random_state_dict(0), max_frames=B * V, device=dev)
    # the weights live once on rank 0; ship them over RCCL (xGMI) and re-derive each rank's
    # graph copies (the only start-up collective)
    est.backbone.sync_weights(src=0)
    cams = syn.make_rig(V, seed=1)
    pipe = MultiViewPipeline(syn.reference_camera_params(cams), estimator=est, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    frames = torch.randint(0, 256, (B, V, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)
    out = {}

    def step():
        o = pipe.process(frames, out, overlap_moments=True)  # moments beside the next backbone
        mdist.gather_frames(o["kpts_3d"], world * B)   # per-step 3D joints to rank 0 (204 B/frame)
        return o

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rank_ms = [1e3 * elapsed / args.steps]
    rccl_world = 1
    if world > 1:
        # every rank's own step time to rank 0 (shows a lagging rank), then the max = the job's time
        rccl_world = torch.distributed.get_world_size()
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        parts = [torch.empty_like(t) for _ in range(rccl_world)]
        torch.distributed.all_gather(parts, t)
        rank_ms = [1e3 * float(p.item()) / args.steps for p in parts]
        elapsed = max(float(p.item()) for p in parts)

    # ---- per-kernel timing with HIP events on the launch stream (not part of the timed region)
    s = torch.cuda.current_stream(dev)
    crops = est.crops[: 2 * B * V]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = max(3, args.steps // 2)
    e[0].record(s)
    for _ in range(reps):
        est.backbone.forward(crops, out=est.heatmaps[: 2 * B * V])
    e[1].record(s)
    torch.cuda.synchronize()
    bb_ms = e[0].elapsed_time(e[1]) / reps
    flops = 2.0 * est.backbone.macs_per_crop() * crops.shape[0]
    bb_tflops = flops / (bb_ms * 1e-3) / 1e12
    extra = {}
    if rank == 0:
        traffic_all, _ = committed_traffic()
        extra["stages"] = stage_lines(est, frames.reshape(B * V, 720, 1280, 3), traffic_all)
        del frames
        torch.cuda.empty_cache()
        if V == 2:
            tri = tri_line(ops, syn, dev, s, V, ops.TRI_REFERENCE, tolerance=True)
            tri["kernel"] = "triangulate_tol2_kernel (+ triangulate_tol2_fallback_kernel)"
            tri["valu_issue"] = tri_valu_issue(tri["avg_launch_ms"], TRI_TOL_PMC)
            tri["solver"] = "tolerance (MVP_TRI_TOLERANCE): the pipeline's default"
            compat = tri_line(ops, syn, dev, s, V, ops.TRI_REFERENCE)
            compat["kernel"] = "triangulate_reference_kernel"
            compat["valu_issue"] = tri_valu_issue(compat["avg_launch_ms"], TRI_REF_PMC)
            tri["reference_compat"] = compat
        else:
            tri = tri_line(ops, syn, dev, s, V, ops.TRI_REFERENCE)
            tri["kernel"] = "triangulate_reference_kernel"
            tri["valu_issue"] = tri_valu_issue(tri["avg_launch_ms"], TRI_REF_PMC)
        extra["roofline_triangulate"] = tri
        if not args.no_extra:
            t4 = tri_line(ops, syn, dev, s, 4, ops.TRI_ALL_VIEWS)
            t4["kernel"] = "triangulate_all_views_kernel"
            t4["config"] = "BASELINE config 3: 4-cam overdetermined 8x4 DLT, all views"
            extra["roofline_triangulate_v4"] = t4
            extra["sgd"] = sgd_line(dev)
            extra["sgd_extrinsic"] = extrinsic_line(dev)
            extra["host_ingest"] = ingest_line(est, V)
            extra["video_decode"] = video_decode_line()
            extra["detector"] = detector_line(dev, est, syn.reference_camera_params(cams), V)

    if rank == 0:
        traffic, traffic_src = committed_traffic()
        total_frames = world * B * args.steps
        res = {
            "metric": METRIC,
            "value": total_frames / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded uint8 1280x720 frames, random-init HRNet-W32 weights, synthetic camera rig)",
            "config": {"workload": f"BASELINE config 2: {V}-cam HRNet-W32 256x192 bf16 (flip test) + batched "
                                   f"4x4 DLT-SVD triangulation", "frames_per_step_per_gpu": B, "views": V,
                       "crops_per_step_per_gpu": 2 * B * V, "parallelism": f"dp{world} (frame-sharded)"},
            "rccl_world": rccl_world,
            "rank_ms_per_step": {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms},
            "roofline": {"bound": "mfma", "kernel": "HRNet-W32 conv graph (one graph forward = one launch)",
                         "achieved": bb_tflops, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": bb_tflops / BF16_PEAK_TFLOPS,
                         "traffic": traffic.get("backbone", {}).get("hbm_bytes_per_launch"),
                         "traffic_source": traffic_src, "flops_per_launch": flops, "avg_launch_ms": bb_ms,
                         "breakdown_source": BREAKDOWN_FILE},
        }
        res.update(extra)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample_frames, args.cpu_sample_frames_1t, V)
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
