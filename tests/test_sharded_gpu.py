"""GPU: BASELINE config 4's per-rank work — one rank's 12.5k-frame shard of the
100k-frame 2-camera stream (8 ranks) through dist.process_sharded at world 1,
chunked through the pipeline's 256-frame batches (ragged last chunk), with the
frames generated on the device per chunk (the stream is 69 GB of uint8).
Checks: shapes/dtypes of the gathered outputs; every frame's kpts_3d against the
oracle triangulation of the GPU's own kpts_2d (cv_ref, <= 1e-4); a re-run of two
chunks (first, ragged last) reproduces the streamed outputs bit for bit."""
import numpy as np
import pytest
import torch

from oracle import cv_ref

pytestmark = pytest.mark.gpu

N_TOTAL, WORLD = 100_000, 8
CHUNK = 256


def _frames(c0, c1, dev):
    g = torch.Generator(device=dev).manual_seed(7919 + c0)
    return torch.randint(0, 256, (c1 - c0, 2, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)


def test_one_rank_shard_of_config4():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import dist as mdist, pipeline, synthetic as syn
    a, b = mdist.shard(N_TOTAL, WORLD, 0)
    n = b - a
    assert n == 12_500
    cams = syn.make_rig(2, seed=1)
    cp = syn.reference_camera_params(cams)
    p = pipeline.MultiViewPipeline(cp, max_frames=2 * CHUNK, seed=0)
    dev = p.device

    def process(s, e):
        outs = {"kpts_2d": [], "heatmaps_2d": [], "kpts_3d": []}
        for c0 in range(s, e, CHUNK):
            o = p.process(_frames(c0, min(e, c0 + CHUNK), dev))
            for k in outs:
                outs[k].append(o[k].clone())
        return {k: torch.cat(v) for k, v in outs.items()}

    full = mdist.process_sharded(process, n)
    torch.cuda.synchronize()
    assert full["kpts_2d"].shape == (n, 17, 3, 2) and full["kpts_3d"].shape == (n, 17, 3)
    assert full["heatmaps_2d"].dtype == torch.float64
    k2 = full["kpts_2d"].cpu().numpy()
    k3 = full["kpts_3d"].cpu().numpy()
    assert np.isfinite(k2).all()
    ref = cv_ref.get_pose_3D(cp, k2, camera_indices=[0, 1])
    np.testing.assert_allclose(k3, ref, rtol=1e-5, atol=1e-4, equal_nan=True)
    for c0 in (0, (n // CHUNK) * CHUNK):
        c1 = min(n, c0 + CHUNK)
        o = p.process(_frames(c0, c1, dev))
        torch.cuda.synchronize()
        for k in ("kpts_2d", "heatmaps_2d", "kpts_3d"):
            assert torch.equal(torch.nan_to_num(o[k]), torch.nan_to_num(full[k][c0:c1])), (c0, k)
