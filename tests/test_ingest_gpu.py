"""GPU: the overlapped host frame supply (pose_estimation.FrameStreamer: pinned staging
filled by a host thread, H2D on a copy stream, double-buffered device frames) gives the
same kpts_2d / heatmaps as feeding each chunk straight to the estimator — for a ragged
frame count (last chunk partial), from in-memory recordings and from .npy files
through run_pose_est (the reference's [0, -1] slice drops the last frame)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_streamer_matches_direct_runs(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    from mvpose.estimator import BatchPoseEstimator
    from mvpose.pose_estimation import FrameStreamer, run_pose_est
    rng = np.random.default_rng(3)
    T, V, H, W = 37, 2, 720, 1280
    base = rng.integers(0, 256, (7, H, W, 3), dtype=np.uint8)
    stacks = [np.ascontiguousarray(base[rng.integers(0, 7, T)]) for _ in range(V)]
    est = BatchPoseEstimator(hrnet.random_state_dict(71), max_frames=16, swap_rb=False)
    kp, hm = FrameStreamer(est, V, (H, W), batch_frames=8).run(stacks)
    torch.cuda.synchronize()
    kp, hm = kp.cpu().numpy(), hm.cpu().numpy()
    for t0 in range(0, T, 8):
        t1 = min(T, t0 + 8)
        fr = torch.tensor(np.stack([np.stack([s[t] for s in stacks]) for t in range(t0, t1)]), device="cuda")
        kt = torch.empty((t1 - t0, 17, 3, V), device="cuda")
        r = est.run(fr.reshape(-1, H, W, 3), n_views=V, kpts_tkv=kt)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(kp[t0:t1], kt.cpu().numpy())
        np.testing.assert_array_equal(hm[t0:t1], r["gaussians"].reshape(t1 - t0, V, 17, 6).cpu().numpy())
    paths = {}
    for v in range(V):
        paths[v] = str(tmp_path / f"cam{v}.npy")
        np.save(paths[v], stacks[v])
    k2, h2 = run_pose_est(est, recording_paths=paths, batch_frames=8)
    assert k2.shape == (T - 1, 17, 3, V)                       # [0, -1] drops the last frame
    np.testing.assert_array_equal(k2, kp[: T - 1])
    np.testing.assert_array_equal(h2, hm[: T - 1])
