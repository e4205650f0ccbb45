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
TRI_T = 100_000             # frames per triangulation-roofline launch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=256, help="synchronised frames per step per GPU")
    ap.add_argument("--views", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frames", type=int, default=12)
    return ap.parse_args()


def committed_traffic():
    """HBM bytes per launch from the newest committed PMC pass (profiles/rNN_traffic.json,
    tools/pmc_traffic.py: 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected) — PMC counters cannot be
    read from inside a normal run."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return {}, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", local if world > 1 else 0)


def cpu_baseline(n_frames, views, seed=0):
    """The reference-equivalent CPU path (oracle restatement):
    torch-CPU fp32 HRNet-W32 at batch 1 per camera with flip test, numpy decode,
    revert + moments, OpenCV-semantics triangulation — timed on this host."""
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
            k, s, _ = heatmap_ref.msra_decode(avg[0].numpy())
            kpts[t, :, :2, v] = heatmap_ref.keypoints_to_image(k, center, scale)
            kpts[t, :, 2, v] = s
            heatmap_ref.heatmap_means_cov_f64(heatmap_ref.warp_affine_linear_f32(avg[0].numpy(), Mh, 720, 1280))
    cv_ref.get_pose_3D(cp, kpts, camera_indices=[0, 1])
    dt = time.perf_counter() - t0
    return {"value": n_frames / dt, "unit": "frames/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n_frames} synthetic {views}-cam 1280x720 frames, batch 1 per camera, flip test, "
                      f"{dt:.1f} s (oracle/ restatement: torch-CPU fp32 HRNet-W32 + numpy decode/revert/moments "
                      f"+ OpenCV-4.9-semantics triangulation in C)"}


def tri_valu_issue(tri_ms):
    """The triangulation kernel's real bound: FP64 VALU issue (OpenCV-order fp64
    undistortion + QR).  From the committed PMC pass (profiles/r01_tri_pmc.json):
    VALU instructions per launch x 4 cycles (wave64 on a 16-lane SIMD) over 1024
    SIMDs at 2.4 GHz = the issue floor; frac = floor / measured launch time."""
    path = os.path.join(ROOT, "profiles", "r01_tri_pmc.json")
    if not os.path.exists(path):
        return None
    pmc = json.load(open(path))
    floor = pmc["valu_issue_floor_ms"]
    return {"valu_instr_per_launch": pmc["valu_instr_per_launch"], "issue_floor_ms": floor,
            "frac": floor / tri_ms, "source": "profiles/r01_tri_pmc.json"}


def main():
    args = parse()
    world, rank, dev = setup_dist(args)
    from mvpose import dist as mdist, hrnet, ops, synthetic as syn
    from mvpose.estimator import BatchPoseEstimator
    from mvpose.pipeline import MultiViewPipeline

    B, V = args.frames, args.views
    sd = hrnet.random_state_dict(0) if rank == 0 or world == 1 else hrnet.random_state_dict(0)
    est = BatchPoseEstimator(sd, max_frames=B * V, device=dev)
    # weights live once on rank 0; ship them over RCCL (xGMI) — the only start-up collective
    mdist.broadcast_([est.backbone.w_dev, est.backbone.f_dev], src=0)
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
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()

    # ---- per-kernel timing with HIP events on the launch stream (not part of the timed region)
    s = torch.cuda.current_stream(dev)
    crops = est.crops[: 2 * B * V]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    reps = max(3, args.steps // 2)
    e[0].record(s)
    for _ in range(reps):
        est.backbone.forward(crops, out=est.heatmaps[: 2 * B * V])
    e[1].record(s)
    # triangulation roofline on a resident stream of TRI_T synchronised frames (BASELINE config 4's
    # 100k-frame stream; one launch = TRI_T*17 problems) — the per-step launch (B frames) is
    # latency-bound and says nothing about the kernel
    kst = syn.make_kpts_2d(syn.make_poses(2000, seed=2), cams, seed=3)
    kst = np.ascontiguousarray(np.tile(kst, (TRI_T // kst.shape[0] + 1, 1, 1, 1))[:TRI_T])
    kst = torch.tensor(kst, device=dev)
    tri_out = torch.empty((TRI_T, 17, 3), dtype=torch.float32, device=dev)
    for _ in range(2):
        ops.triangulate(kst, pipe.cams, [0, 1], out=tri_out)
    tri_reps = 200  # ~13 ms: shorter windows swing +-15 % with the clock state
    e[2].record(s)
    for _ in range(tri_reps):
        ops.triangulate(kst, pipe.cams, [0, 1], out=tri_out)
    e[3].record(s)
    torch.cuda.synchronize()
    bb_ms = e[0].elapsed_time(e[1]) / reps
    tri_ms = e[2].elapsed_time(e[3]) / tri_reps
    flops = 2.0 * est.backbone.macs_per_crop() * crops.shape[0]
    bb_tflops = flops / (bb_ms * 1e-3) / 1e12
    tri_bytes = 12.0 * 17 * (V + 1) * TRI_T  # read x,y,conf per view + write xyz per joint
    tri_gbs = tri_bytes / (tri_ms * 1e-3) / 1e9

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
            "roofline": {"bound": "mfma", "kernel": "HRNet-W32 conv graph (tconv/wsconv/basic_block/conv_mfma "
                                                    "kernels, one graph forward = one launch)",
                         "achieved": bb_tflops, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": bb_tflops / BF16_PEAK_TFLOPS,
                         "traffic": traffic.get("backbone", {}).get("hbm_bytes_per_launch"),
                         "traffic_source": traffic_src, "flops_per_launch": flops, "avg_launch_ms": bb_ms},
            "roofline_triangulate": {"bound": "hbm", "kernel": "triangulate_reference_kernel",
                                     "workload": f"{TRI_T} resident synchronised {V}-cam frames per launch "
                                                 f"(BASELINE config 4 stream)",
                                     "achieved": tri_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": tri_gbs / HBM_PEAK_GBS, "bytes_per_launch": tri_bytes,
                                     "frames_per_s": TRI_T / (tri_ms * 1e-3), "avg_launch_ms": tri_ms,
                                     "valu_issue": tri_valu_issue(tri_ms)},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample_frames, V)
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
