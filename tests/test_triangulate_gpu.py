"""GPU parity: HIP triangulation (mvp_triangulate) vs the oracle and the
reference's golden vectors.

BASELINE north_star bound: 1e-4 mm.  World units are cm here (the reference's calibration
units), so the bound is 1e-5 world units — below one float32 ulp (3.05e-5 cm) at
the rigs' ~350 cm: at these magnitudes the north_star bound means BIT-IDENTICAL float32
outputs, and that is what every solver is held to: the exact path (Jacobi restatement) against
the oracle, and the default (QR, certified) and tolerance (normal equations, certified)
solvers against the exact path, on every point (NaN where it is NaN).  utils.DLT is a
different algorithm (numpy SVD of AᵀA): its known answers keep a 1e-4 world-unit tolerance."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import cv_ref
from mvpose import synthetic as syn

pytestmark = pytest.mark.gpu
ATOL = 1e-4


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import ops as _ops
    return _ops


def _cams(d):
    return {i: [d["K"][i], d["R"][i], d["T"][i], d["dist"][i]] for i in range(d["K"].shape[0])}


def _run(ops, cp, kpts, ci, mode=0, ignore_dist=False):
    if ignore_dist:
        cp = {k: [K, R, T, np.asarray(dist) * 0] for k, (K, R, T, dist) in cp.items()}
    cams = torch.tensor(ops.pack_cameras(cp), device="cuda")
    k = torch.tensor(np.ascontiguousarray(kpts), device="cuda")
    out = ops.triangulate(k, cams, ci, mode=mode)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _check(out, ref):
    """Bit-identical float32 (NaN where the reference is NaN)."""
    assert out.shape == ref.shape and out.dtype == ref.dtype
    same = (out == ref) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), (f"{(~same).sum()} of {same.size} outputs differ from the reference, max |d| "
                        f"{np.nanmax(np.abs(out - ref)):.3g}")


@pytest.mark.parametrize("tag,ci,ign", [("01", [0, 1], False), ("012", [0, 1, 2], False),
                                        ("12", [1, 2], False), ("01_nodist", [0, 1], True)])
def test_golden_get_pose_3D(ops, tag, ci, ign):
    """The reference's own get_pose_3D output (its cv2 leaves = the oracle's restatement):
    default and exact solvers bit-identical."""
    d = np.load(os.path.join(GOLDEN, "pose3d_select.npz"))
    _check(_run(ops, _cams(d), d["kpts"], ci, ignore_dist=ign), d["out_" + tag])
    _check(_run(ops, _cams(d), d["kpts"], ci, mode=ops.TRI_REFERENCE | ops.TRI_EXACT_JACOBI, ignore_dist=ign),
           d["out_" + tag])


def test_golden_dlt(ops):
    d = np.load(os.path.join(GOLDEN, "dlt_kat.npz"))
    out = _run(ops, _cams(d), d["kpts"], [0, 1]).reshape(-1, 3)
    np.testing.assert_allclose(out, d["out"], rtol=0, atol=ATOL)


@pytest.mark.parametrize("V,T,seed", [(2, 300, 1), (3, 100, 2), (8, 50, 3)])
def test_seeded_vs_oracle(ops, V, T, seed):
    cams = syn.make_rig(V, seed=seed)
    k = syn.make_kpts_2d(syn.make_poses(T, seed=seed + 10), cams, seed=seed + 20)
    cp = syn.reference_camera_params(cams)
    ref = cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1])
    _check(_run(ops, cp, k, [0, 1]), ref)


def test_top2_of_many(ops):
    cams = syn.make_rig(5, seed=4)
    k = syn.make_kpts_2d(syn.make_poses(40, seed=5), cams, seed=6)
    k[::3, ::2, 2, 3] = k[::3, ::2, 2, 1]  # ties
    k[5, 3, 2, 2] = np.nan
    cp = syn.reference_camera_params(cams)
    ci = [0, 1, 2, 3, 4]
    ref = cv_ref.get_pose_3D(cp, k, camera_indices=ci)
    _check(_run(ops, cp, k, ci), ref)


def test_nan_and_empty(ops):
    cams = syn.make_rig(2, seed=7)
    k = syn.make_kpts_2d(syn.make_poses(4, seed=8), cams, seed=9)
    k[1, 2, 0, 0] = np.nan
    k[2, 5, 1, 1] = np.nan
    cp = syn.reference_camera_params(cams)
    ref = cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1])
    out = _run(ops, cp, k, [0, 1])
    assert np.isnan(out[1, 2]).all() and np.isnan(ref[1, 2]).all()
    _check(out, ref)
    empty = _run(ops, cp, np.zeros((0, 17, 3, 2), np.float32), [0, 1])
    assert empty.shape == (0, 17, 3)


@pytest.mark.parametrize("V", [2, 4, 8])
def test_all_views_vs_oracle(ops, V):
    cams = syn.make_rig(V, seed=11 + V)
    k = syn.make_kpts_2d(syn.make_poses(60, seed=12), cams, seed=13)
    cp = [(c["K"], c["R"], c["T"], c["dist"]) for c in cams]
    ci = list(range(V))
    ref = cv_ref.triangulate_all_views(cp, k, ci)
    _check(_run(ops, syn.reference_camera_params(cams), k, ci, mode=ops.TRI_ALL_VIEWS), ref)


@pytest.mark.parametrize("V,mode,noise", [(2, 0, 1.0), (2, 0, 0.0), (2, 0, 40.0), (4, 1, 1.0), (8, 1, 3.0)])
def test_fast_solver_matches_exact_jacobi(ops, V, mode, noise):
    """QR + inverse-iteration null vector (default, certified) vs the exact JacobiSVDImpl_
    restatement on the same inputs: bit-identical, including noise-free (exactly singular A)
    and badly inconsistent (40 px) views; the exact path also equals the oracle bit for bit."""
    cams = syn.make_rig(V, seed=31 + V)
    k = syn.make_kpts_2d(syn.make_poses(3000, seed=32), cams, seed=33, noise_px=noise)
    cp = syn.reference_camera_params(cams)
    ci = list(range(V)) if mode == ops.TRI_ALL_VIEWS else [0, 1]
    cams_d = torch.tensor(ops.pack_cameras(cp), device="cuda")
    kd = torch.tensor(k, device="cuda")
    fast = ops.triangulate(kd, cams_d, ci, mode=mode).cpu().numpy()
    exact = ops.triangulate(kd, cams_d, ci, mode=mode, exact=True).cpu().numpy()
    _check(fast, exact)
    if mode == ops.TRI_ALL_VIEWS:
        ref = cv_ref.triangulate_all_views([(c["K"], c["R"], c["T"], c["dist"]) for c in cams], k, ci)
    else:
        ref = cv_ref.get_pose_3D(cp, k, camera_indices=ci)
    _check(exact, ref)


def test_fast_solver_degenerate_inputs(ops):
    """Random (geometrically inconsistent) 2D points and NaNs: the fallback must
    reproduce the exact path."""
    cams = syn.make_rig(2, seed=41)
    rng = np.random.default_rng(42)
    k = np.zeros((500, 17, 3, 2), np.float32)
    k[:, :, 0] = rng.uniform(0, 1280, (500, 17, 2))
    k[:, :, 1] = rng.uniform(0, 720, (500, 17, 2))
    k[:, :, 2] = rng.uniform(0.3, 1, (500, 17, 2))
    k[7, 3, 0, 1] = np.nan
    k[9, 4, 1, 0] = np.inf
    cp = syn.reference_camera_params(cams)
    cams_d = torch.tensor(ops.pack_cameras(cp), device="cuda")
    kd = torch.tensor(k, device="cuda")
    fast, fw = (t.cpu().numpy() for t in ops.triangulate(kd, cams_d, [0, 1], return_xyzw=True))
    exact, ew = (t.cpu().numpy() for t in ops.triangulate(kd, cams_d, [0, 1], exact=True, return_xyzw=True))
    ref = cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1])
    _check(exact, ref)
    _check(fast, exact)
    # the null vectors agree up to sign; X = v/w is compared where w is not ~0 (points at infinity)
    fw, ew = fw.reshape(-1, 4), ew.reshape(-1, 4)
    ok = np.isfinite(ew).all(1)
    assert np.array_equal(ok, np.isfinite(fw).all(1))
    sgn = np.sign(np.sum(fw[ok] * ew[ok], axis=1, keepdims=True))
    np.testing.assert_allclose(fw[ok] * sgn, ew[ok], rtol=0, atol=1e-9)
    far = np.abs(ew[:, 3]) < 1e-6
    sel = ok & ~far
    np.testing.assert_allclose(fast.reshape(-1, 3)[sel], exact.reshape(-1, 3)[sel], rtol=1e-5, atol=ATOL)


def test_full_size_roundtrip_property(ops):
    """BASELINE config 4 size (100k frames x 17 joints, V=2): noise-free
    projections must triangulate back to the poses; order of the two cameras
    must not matter beyond f32 rounding."""
    cams = syn.make_rig(2, seed=21)
    T = 100_000
    poses = syn.make_poses(T, seed=22)
    k = syn.make_kpts_2d(poses, cams, seed=23, noise_px=0.0)
    cp = syn.reference_camera_params(cams)
    out = _run(ops, cp, k, [0, 1])
    assert np.isfinite(out).all()
    np.testing.assert_allclose(out, poses, atol=2e-3)
    k2 = k.copy()
    k2[:, :, 2, :] = k[:, :, 2, ::-1]  # flip the confidence order -> swapped camera order
    out2 = _run(ops, cp, k2, [0, 1])
    np.testing.assert_allclose(out2, out, atol=ATOL)


# ------------------------------------------------------------------ tolerance mode
def _tol_vs_exact(ops, cp, k, ci=(0, 1)):
    cams_d = torch.tensor(ops.pack_cameras(cp), device="cuda")
    kd = torch.tensor(np.ascontiguousarray(k), device="cuda")
    tol = ops.triangulate(kd, cams_d, list(ci), tolerance=True).cpu().numpy()
    ex = ops.triangulate(kd, cams_d, list(ci), exact=True).cpu().numpy()
    return tol, ex


def _fallbacks(ops, fn):
    before = ops.triangulate_fallback_total()
    r = fn()
    return r, ops.triangulate_fallback_total() - before


@pytest.mark.parametrize("seed,noise", [(51, 1.0), (52, 0.0), (53, 40.0), (54, 3.0)])
def test_tolerance_mode_vs_exact(ops, seed, noise):
    """MVP_TRI_TOLERANCE (mixed f32/fp64 undistortion + normal-equation inverse iteration,
    certified per point) vs the exact-rounding restatement on the same points: bit-identical
    on every coordinate (the north_star's 1e-4 mm = 1e-5 cm is below one f32 ulp here) —
    noise-free (singular A), 1-3 px and badly inconsistent (40 px) views; the exact path
    equals the oracle."""
    cams = syn.make_rig(2, seed=seed)
    k = syn.make_kpts_2d(syn.make_poses(3000, seed=seed + 1), cams, seed=seed + 2, noise_px=noise)
    cp = syn.reference_camera_params(cams)
    (tol, ex), nfb = _fallbacks(ops, lambda: _tol_vs_exact(ops, cp, k))
    print(f"tolerance vs exact (noise {noise} px): {nfb} of {k.shape[0] * 17} points re-solved on the exact path, "
          f"max |d| {np.nanmax(np.abs(tol - ex)):.3g}")
    _check(tol, ex)
    _check(ex, cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1]))


@pytest.mark.parametrize("tag,ign", [("01", False), ("01_nodist", True)])
def test_tolerance_mode_golden(ops, tag, ign):
    """The reference's own get_pose_3D golden vectors (pose3d_select.npz), camera_indices [0, 1]."""
    d = np.load(os.path.join(GOLDEN, "pose3d_select.npz"))
    cp = _cams(d)
    if ign:
        cp = {k: [K, R, T, np.asarray(dist) * 0] for k, (K, R, T, dist) in cp.items()}
    cams = torch.tensor(ops.pack_cameras(cp), device="cuda")
    out = ops.triangulate(torch.tensor(d["kpts"], device="cuda"), cams, [0, 1], tolerance=True).cpu().numpy()
    _check(out, d["out_" + tag])


def test_tolerance_mode_ties_nans_degenerate(ops):
    """Equal confidences (np.argsort keeps [0, 1]), NaN / Inf coordinates and confidences,
    geometrically inconsistent random points (incl. points at infinity): the exact path's bits
    everywhere, and the exact path equals the oracle."""
    cams = syn.make_rig(2, seed=61)
    rng = np.random.default_rng(62)
    k = syn.make_kpts_2d(syn.make_poses(400, seed=63), cams, seed=64)
    k[::4, :, 2, 1] = k[::4, :, 2, 0]                       # ties
    k[5, 3, 2, 0] = np.nan                                  # NaN confidence sorts last
    k[6, 4, 2, 1] = np.nan
    k[7, 3, 0, 1] = np.nan
    k[9, 4, 1, 0] = np.inf
    k[200:] = 0
    k[200:, :, 0] = rng.uniform(0, 1280, (200, 17, 2))      # random, inconsistent views
    k[200:, :, 1] = rng.uniform(0, 720, (200, 17, 2))
    k[200:, :, 2] = rng.uniform(0.3, 1, (200, 17, 2))
    cp = syn.reference_camera_params(cams)
    (tol, ex), nfb = _fallbacks(ops, lambda: _tol_vs_exact(ops, cp, k))
    print(f"ties / NaN / random views: {nfb} of {k.shape[0] * 17} points re-solved on the exact path")
    _check(ex, cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1]))
    _check(tol, ex)


def test_tolerance_mode_full_size(ops):
    """BASELINE config 4 size (100 k frames x 17 joints): tolerance vs exact bit-identical on
    every coordinate (0.5 px noise; 1.7 M points), the default solver too, and noise-free
    projections triangulate back to the poses (f32 pixel rounding only)."""
    cams = syn.make_rig(2, seed=71)
    cp = syn.reference_camera_params(cams)
    poses = syn.make_poses(100_000, seed=72)
    k = syn.make_kpts_2d(poses, cams, seed=73, noise_px=0.5)
    (tol, ex), nfb = _fallbacks(ops, lambda: _tol_vs_exact(ops, cp, k))
    print(f"100k frames: {nfb} of {k.shape[0] * 17} points ({nfb / (k.shape[0] * 17):.2e}) re-solved on the exact "
          f"path, max |d| {np.abs(tol - ex).max():.3g}")
    assert np.isfinite(tol).all()
    _check(tol, ex)
    _check(_run(ops, cp, k, [0, 1]), ex)
    k0 = syn.make_kpts_2d(poses[:10_000], cams, seed=73, noise_px=0.0)
    tol0, ex0 = _tol_vs_exact(ops, cp, k0)
    err = np.abs(tol0 - poses[:10_000])
    print(f"noise-free 10k: max |tol - pose| {err.max():.3g}")
    _check(tol0, ex0)
    np.testing.assert_allclose(tol0, poses[:10_000], rtol=0, atol=2e-2)


@pytest.mark.parametrize("origin", [True, False])
def test_tolerance_mode_rig_without_origin_camera(ops, origin):
    """The closed-form rows of the camera at the world origin (P = [K | 0]) vs a rig where no
    camera sits there (the whole rig moved and rotated): bit-identical to the exact path both
    ways, and to the oracle."""
    cams = syn.make_rig(2, seed=75)
    if not origin:
        th = 0.3
        Rw = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
        tw = np.array([[12.0], [-7.0], [30.0]])
        for c in cams:   # X_cam = R (Rw^T (X' - tw)) + T for world points X' = Rw X + tw
            c["T"] = c["T"] - c["R"] @ Rw.T @ tw
            c["R"] = c["R"] @ Rw.T
    cp = syn.reference_camera_params(cams)
    k = syn.make_kpts_2d(syn.make_poses(2000, seed=76), syn.make_rig(2, seed=75), seed=77, noise_px=1.0)
    (tol, ex), nfb = _fallbacks(ops, lambda: _tol_vs_exact(ops, cp, k))
    print(f"origin camera {origin}: {nfb} of {k.shape[0] * 17} points re-solved on the exact path")
    _check(tol, ex)
    _check(ex, cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1]))


@pytest.mark.parametrize("frames", [1000, 6000])
def test_tolerance_mode_fallback_list_and_sweep(ops, frames, monkeypatch):
    """The tolerance kernel's out-of-line fallback: with every point forced onto it the result
    is the exact path's, bit for bit — through the per-stream list (1,000 frames = 17 k points)
    and, past the list's 65,536 entries, through the sentinel sweep (6,000 frames = 102 k
    points); the next unforced launch on the same stream starts from an empty list."""
    cams = syn.make_rig(2, seed=81)
    k = syn.make_kpts_2d(syn.make_poses(frames, seed=82), cams, seed=83, noise_px=1.0)
    k[3, 2, 0, 0] = np.nan
    cp = syn.reference_camera_params(cams)
    cams_d = torch.tensor(ops.pack_cameras(cp), device="cuda")
    kd = torch.tensor(np.ascontiguousarray(k), device="cuda")
    ex, exw = ops.triangulate(kd, cams_d, [0, 1], exact=True, return_xyzw=True)
    monkeypatch.setenv("MVPOSE_TRI_FORCE_FALLBACK", "1")
    fo, fow = ops.triangulate(kd, cams_d, [0, 1], tolerance=True, return_xyzw=True)
    monkeypatch.delenv("MVPOSE_TRI_FORCE_FALLBACK")
    np.testing.assert_array_equal(fo.cpu().numpy(), ex.cpu().numpy())
    np.testing.assert_array_equal(fow.cpu().numpy(), exw.cpu().numpy())
    tol = ops.triangulate(kd, cams_d, [0, 1], tolerance=True).cpu().numpy()
    _check(tol, ex.cpu().numpy())


def test_tolerance_mode_two_host_threads_one_stream(ops, monkeypatch):
    """Two host threads triangulating different-size batches on the same (default) stream with
    every point forced onto the fallback list: each call's list launch pair is enqueued under
    the list's lock, so neither call re-solves the other's indices (A_tol, B_tol,
    A_fb, B_fb would read B's indices with A's pointers) and both equal the exact path."""
    import threading
    cams = syn.make_rig(2, seed=91)
    cp = syn.reference_camera_params(cams)
    cams_d = torch.tensor(ops.pack_cameras(cp), device="cuda")
    ks = [torch.tensor(syn.make_kpts_2d(syn.make_poses(n, seed=92 + n), cams, seed=93, noise_px=1.0), device="cuda")
          for n in (300, 2000)]
    exact = [ops.triangulate(k, cams_d, [0, 1], exact=True).cpu().numpy() for k in ks]
    monkeypatch.setenv("MVPOSE_TRI_FORCE_FALLBACK", "1")
    outs = [[], []]
    errs = []

    def work(i):
        try:
            torch.cuda.set_device(0)
            for _ in range(20):
                outs[i].append(ops.triangulate(ks[i], cams_d, [0, 1], tolerance=True))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    monkeypatch.delenv("MVPOSE_TRI_FORCE_FALLBACK")
    assert not errs, errs
    for i in range(2):
        for o in outs[i]:
            np.testing.assert_array_equal(o.cpu().numpy(), exact[i])


def _adversarial_rig(baseline, seed):
    """Camera 0 at the origin, camera 1 displaced by `baseline` cm sideways and slightly forward,
    both looking at the subject: a tiny baseline makes the rays nearly parallel (sigma_4 close to
    sigma_3 in A, the regime the empirical certification constants were not fitted on)."""
    rng = np.random.default_rng(seed)
    cams = syn.make_rig(2, seed=seed)
    pos = np.array([baseline, rng.uniform(-0.1, 0.1) * baseline, 0.05 * baseline])
    R, T = syn._look_at(pos, syn.SUBJECT_CENTER + np.array([0.0, 0.0, 0.0]))
    cams[1]["R"], cams[1]["T"] = R, T
    return cams


@pytest.mark.parametrize("baseline", [0.05, 0.5, 5.0, 40.0])
def test_tolerance_mode_adversarial_geometry(ops, baseline):
    """the certification bound is empirical, so probe where it is weakest — tiny
    baselines (near-parallel rays, ill-conditioned A), points on and near the baseline (the
    epipoles: the two views see the point at the same spot), points far behind the subject and
    sub-pixel noise.  Tolerance and default solvers stay bit-identical to the exact path, which
    equals the oracle."""
    cams = _adversarial_rig(baseline, seed=81)
    cp = syn.reference_camera_params(cams)
    rng = np.random.default_rng(82)
    poses = syn.make_poses(400, seed=83)
    c1 = -cams[1]["R"].T @ cams[1]["T"].reshape(3)                 # camera 1's centre
    # frames 100-199: joints on the line through both centres (the epipoles) and beyond
    s = rng.uniform(-3.0, 4.0, (100, 17, 1))
    poses[100:200] = s * c1 + rng.normal(0.0, 1e-3 * max(baseline, 1.0), (100, 17, 3)) + np.array([0, 0, 0.5])
    poses[200:300] *= rng.uniform(1.0, 30.0, (100, 17, 1))         # far points (up to ~100 m)
    k = syn.make_kpts_2d(poses, cams, seed=84, noise_px=0.25)
    (tol, ex), nfb = _fallbacks(ops, lambda: _tol_vs_exact(ops, cp, k))
    print(f"baseline {baseline} cm: {nfb} of {k.shape[0] * 17} points re-solved on the exact path")
    _check(ex, cv_ref.get_pose_3D(cp, k, camera_indices=[0, 1]))
    _check(tol, ex)
    _check(_run(ops, cp, k, [0, 1]), ex)
