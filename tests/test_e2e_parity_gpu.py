"""GPU: end-to-end parity on IDENTICAL frames — the bf16 HIP pipeline
(MultiViewPipeline.process: crop, HRNet-W32 bf16 with flip test, decode, moments,
triangulation) against the fp32 oracle path run independently on the same uint8
frames and the same cameras (oracle/heatmap_ref.preprocess -> hrnet_ref
flip_test_forward -> msra_decode / keypoints_to_image -> cv_ref.get_pose_3D), the
reference's pose_estimation.py:88-135 + :319-322 loop.

Two workloads (module fixture `runs`, parametrised):
* "peaked" — the headline parity case: mvpose.hrnet.peaked_state_dict (seeded random
  convolutions with BatchNorms, stem, last high-resolution branch and head fitted on
  rendered skeleton frames, tools/train_peaked_hrnet.py) on synthetic.make_skeleton_frames:
  one trained-model-like peak per joint, so argmax parity is measured on decidable maps;
* "random" — random_state_dict's activation-stable seeded weights on uniform-noise frames:
  O(0.1) maps, many without any peak, so most argmaxes are near-ties (a pessimistic figure).
bf16 weights/activations through ~90 layers move the heatmaps by ~1e-2 relative, so an
argmax can only move where two cells are within that of each other.
Asserted per workload (tolerances in LIMITS; measured rates printed and recorded in DESIGN §5):
* argmax agreement >= argmax_min of all (frame, view, joint) heatmaps;
* >= decidable_fraction of maps lead their runner-up by > MARGIN of the map's max|h| in
  fp32, and there the argmax agrees on >= decidable_min;
* where the argmax agrees (and the max's sign, which decides MSRA's -1 marker), the decoded
  keypoint equals the oracle's, except by the +-0.25-cell MSRA refinement step (one or two
  steps) only on an axis where the oracle's own sign(h[x+1] - h[x-1]) is a near-tie
  (|h[x+1] - h[x-1]| <= MARGIN x max|h|: bf16 cannot decide it), and is bit-exact on
  >= exact_min of those maps;
* where both views' x, y are bit-exact and the camera order (ascending score, the
  reference's top-2 rule) agrees, kpts_3d is bit-identical (the north_star's 1e-4 mm is
  below one float32 ulp in cm) — on >= k3_min of all joints.
"""
import numpy as np
import pytest
import torch

from oracle import cv_ref, heatmap_ref, hrnet_ref

pytestmark = pytest.mark.gpu

V = 2
FRAMES = {"peaked": 128, "random": 32}   # synchronised frames per workload (x V camera-frames)
MARGIN = 1e-2              # fp32 top-1 lead over top-2, in units of the map's max|h|
LIMITS = {
    # measured (r04a, MI355X): peaked (128 frames, 4,352 maps) argmax 0.9970, decidable 0.956
    # with agreement 1.000, kpts_2d bit-exact on 0.9882 of same-argmax maps (51 two-step
    # coordinates, all at oracle near-ties), kpts_3d compared on 2081/2176 = 0.956 of joints;
    # random (32 frames, 1,088 maps) argmax 0.838, decidable 0.284 with agreement 0.990,
    # kpts_2d exact 0.998 where the argmax agrees, kpts_3d on 307/544 = 0.564 of joints
    "peaked": dict(argmax_min=0.99, decidable_fraction=0.93, decidable_min=0.99, exact_min=0.97, k3_min=0.92),
    "random": dict(argmax_min=0.80, decidable_fraction=0.20, decidable_min=0.98, exact_min=0.50, k3_min=0.45),
}


@pytest.fixture(scope="module", params=["peaked", "random"])
def runs(request):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet, pipeline, synthetic as syn
    T = FRAMES[request.param]
    if request.param == "peaked":
        sd = hrnet.peaked_state_dict()
        frames = syn.make_skeleton_frames(T * V, seed=31)[0].reshape(T, V, 720, 1280, 3)
    else:
        sd = hrnet.random_state_dict(21)
        frames = syn.make_frames(T * V, seed=31).reshape(T, V, 720, 1280, 3)
    cams = syn.make_rig(V, seed=4)
    cp = syn.reference_camera_params(cams)
    p = pipeline.MultiViewPipeline(cp, max_frames=T * V, state_dict=sd)
    out = p.process(torch.tensor(frames, device="cuda"))
    torch.cuda.synchronize()
    gpu = {k: out[k].cpu().numpy() for k in ("kpts_2d", "heatmaps_2d", "kpts_3d")}
    gpu_avg = p.estimator.avg[: T * V].cpu().numpy()
    # the fp32 oracle path on the same frames
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    model = hrnet_ref.build(sd)
    M, center, scale = heatmap_ref.topdown_crop_matrix(1280, 720)
    k2 = np.zeros((T, 17, 3, V), np.float32)
    amax = np.zeros((T, V, 17), np.int64)
    oavg = np.zeros((T, V, 17, 64 * 48), np.float32)
    flat = frames.reshape(T * V, 720, 1280, 3)
    for c0 in range(0, T * V, 16):        # the oracle network in batches of 16 camera-frames
        xs = torch.from_numpy(np.stack([heatmap_ref.preprocess(f, M) for f in flat[c0:c0 + 16]]))
        avg, _, _ = hrnet_ref.flip_test_forward(model, xs)
        for i in range(avg.shape[0]):
            t, v = divmod(c0 + i, V)
            a = avg[i].numpy()
            oavg[t, v] = a.reshape(17, -1)
            k, s, idx = heatmap_ref.msra_decode(a)
            k2[t, :, :2, v] = heatmap_ref.keypoints_to_image(k, center, scale)
            k2[t, :, 2, v] = s
            amax[t, v] = idx
    k3 = cv_ref.get_pose_3D(cp, k2, camera_indices=[0, 1])
    gam = np.stack([heatmap_ref.msra_decode(gpu_avg[i])[2] for i in range(T * V)]).reshape(T, V, 17)
    return dict(gpu=gpu, k2=k2, k3=k3, amax=amax, gamax=gam, scale=scale, oavg=oavg, name=request.param,
                lim=LIMITS[request.param])


def test_argmax_agreement(runs):
    agree = runs["gamax"] == runs["amax"]
    rate = agree.mean()
    print(f"[{runs['name']}] argmax agreement {rate:.4f} ({agree.sum()}/{agree.size})")
    assert rate >= runs["lim"]["argmax_min"]


def test_argmax_agreement_on_decidable_maps(runs):
    """Where the fp32 oracle's maximum leads its runner-up cell by more than the bf16
    path's own error, the argmax must agree (>= the workload's decidable_min).  The error scale is the
    map's magnitude: bf16 heatmaps differ from fp32 by ~1-3 % of max|h| per map (measured,
    tools/e2e_diag.py), so a lead below MARGIN x max|h| is a near-tie that bf16 compute
    (the allowed dtype) cannot resolve.  Many random-weight maps have no peak at all (all
    cells below zero, the head bias): their argmax is decided by noise in either dtype.
    Agreement there must reach the workload's decidable_min."""
    o = runs["oavg"]                                                     # (T, V, 17, HW)
    top2 = -np.sort(-o, axis=-1)[..., :2]
    lead = (top2[..., 0] - top2[..., 1]) / np.abs(o).max(axis=-1)
    agree = runs["gamax"] == runs["amax"]
    for m in (0.0, 1e-3, 1e-2, 2e-2, 5e-2, 1e-1):
        sel = lead > m
        print(f"[{runs['name']}] lead > {m:g} max|h|: {sel.mean():.3f} of maps, argmax agreement "
              f"{agree[sel].mean() if sel.any() else 1:.4f}")
    sel = lead > MARGIN
    assert sel.sum() >= runs["lim"]["decidable_fraction"] * sel.size, sel.mean()
    assert agree[sel].mean() >= runs["lim"]["decidable_min"], agree[sel].mean()


def _agree(runs):
    """(T, 17, V): same argmax AND the same MSRA validity (a max <= 0 decodes to -1, so a
    score near 0 can flip the keypoint to the invalid marker with the argmax unchanged)."""
    g, o = runs["gpu"]["kpts_2d"], runs["k2"]
    same = (runs["gamax"] == runs["amax"]).transpose(0, 2, 1)
    valid_same = (g[:, :, 2, :] > 0) == (o[:, :, 2, :] > 0)
    print(f"validity flips (score sign) on {(same & ~valid_same).sum()} of {same.sum()} same-argmax maps")
    return same & valid_same


def _refinement_near_tie(runs):
    """(T, 17, 2, V): the oracle's MSRA refinement difference h[x+1] - h[x-1] (x axis) /
    h[y+1] - h[y-1] (y axis) at its argmax is within MARGIN x max|h| of zero."""
    o = runs["oavg"].reshape(runs["oavg"].shape[:3] + (64, 48))         # (T, V, 17, H, W)
    am = runs["amax"]
    py, px = am // 48, am % 48
    T = o.shape[0]
    tie = np.zeros((T, 17, 2, V), bool)
    for t in range(T):
        for v in range(V):
            for j in range(17):
                h = o[t, v, j]
                x, y = px[t, v, j], py[t, v, j]
                lim = MARGIN * np.abs(h).max()
                if 0 < x < 47:
                    tie[t, j, 0, v] = abs(float(h[y, x + 1]) - float(h[y, x - 1])) <= lim
                if 0 < y < 63:
                    tie[t, j, 1, v] = abs(float(h[y + 1, x]) - float(h[y - 1, x])) <= lim
    return tie


def test_keypoints_where_argmax_agrees(runs):
    g, o = runs["gpu"]["kpts_2d"], runs["k2"]
    agree = _agree(runs)                                                 # (T, 17, V)
    step = np.float32(runs["scale"][0]) / np.float32(192.0)              # one 0.25-cell step in image px
    d = np.abs(g[:, :, :2, :] - o[:, :, :2, :])                          # (T, 17, 2, V)
    tie = _refinement_near_tie(runs)
    steps = (np.abs(d - step) <= 1e-3 * step) | (np.abs(d - 2 * step) <= 1e-3 * step)
    ok = (d == 0) | (steps & tie)
    print(f"[{runs['name']}] refinement steps off by one/two on {int(((d > 0) & agree[:, :, None, :]).sum())} "
          f"coordinates, all at oracle near-ties: {bool(ok.transpose(0, 1, 3, 2)[agree].all())}")
    exact = (d == 0).all(axis=2) & agree
    one = ((d > 0) & (d < 1.5 * step)).any(axis=2) & agree
    print(f"[{runs['name']}] kpts_2d bit-exact {exact.mean():.4f} of all, "
          f"{exact.sum() / max(1, agree.sum()):.4f} where argmax agrees; one-step {one.sum()}, "
          f"two-step {(agree.sum() - exact.sum() - one.sum())} of {agree.sum()}")
    assert ok.transpose(0, 1, 3, 2)[agree].all()
    assert exact.sum() >= runs["lim"]["exact_min"] * agree.sum()


def test_kpts_3d_where_inputs_agree(runs):
    """north_star: kpts_3d within 1e-4 mm of the reference triangulation on identical 2D inputs.
    World units are cm, so the bound is 1e-5 cm, below one float32 ulp (~3e-5 cm at
    these ~350 cm coordinates): it means BIT-IDENTICAL.  The pipeline's triangulation is
    certified bit-identical to the OpenCV-4.9 restatement (tests/test_triangulate_gpu.py), so
    wherever both views' x, y are bit-exact and the camera order agrees (np.argsort ascending:
    camera 1 first only when score0 > score1, a tie keeps [0, 1]; pose_estimation.py:32-41),
    kpts_3d is asserted array_equal — anything else is a bug, not rounding."""
    g2, o2 = runs["gpu"]["kpts_2d"], runs["k2"]
    xy_exact = (g2[:, :, :2, :] == o2[:, :, :2, :]).all(axis=(2, 3)) & _agree(runs).all(axis=2)  # (T, 17)
    order_same = (g2[:, :, 2, 0] > g2[:, :, 2, 1]) == (o2[:, :, 2, 0] > o2[:, :, 2, 1])
    sel = xy_exact & order_same
    d = np.abs(runs["gpu"]["kpts_3d"] - runs["k3"])[sel]
    print(f"[{runs['name']}] kpts_3d compared on {sel.sum()}/{sel.size} joints, "
          f"max |d| {np.nanmax(d) if d.size else 0:.3g} cm")
    assert sel.sum() > 0 and sel.sum() >= runs["lim"]["k3_min"] * sel.size
    np.testing.assert_array_equal(runs["gpu"]["kpts_3d"][sel], runs["k3"][sel])
