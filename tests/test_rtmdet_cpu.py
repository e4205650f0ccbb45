"""RTMDet-m person detector (f1): host builder, oracle restatements and wiring, on CPU.

The reference's detector (mmpose_pose_estimation.py:98-99, :234-250; mmdet RTMDet-m,
examples/model_paths.yaml:2-4) is restated in oracle/rtmdet_ref.py; mmdet / mmcv / cv2
are absent, so its parity against them is unpinned.  Here: the product's weight naming
equals the restated modules', the HIP runtime's op list (views, channel padding, BN
folding, fused sibling convs) reproduces the restated network exactly when executed in
fp32 (tests/det_interp.py), and the preprocessing / post-processing restatements behave
as OpenCV / mmcv define them.
"""
import numpy as np
import pytest
import torch

import det_interp
from mvpose import rtmdet as D
from oracle import rtmdet_ref as R


@pytest.fixture(scope="module")
def sd():
    return D.random_state_dict(0)


def test_state_dict_matches_mmdet_module_tree(sd):
    ref = R.RTMDet().state_dict()
    assert set(sd) == set(ref)
    for k, v in ref.items():
        assert tuple(sd[k].shape) == tuple(v.shape), k
    # share_conv: every level's head conv weights equal level 0's
    for br in ("cls", "reg"):
        for i in range(2):
            w0 = sd[f"bbox_head.{br}_convs.0.{i}.conv.weight"]
            for lvl in (1, 2):
                assert torch.equal(sd[f"bbox_head.{br}_convs.{lvl}.{i}.conv.weight"], w0)


def test_macs_rtmdet_m(sd):
    spec, _ = D.build_rtmdet_m(sd, 640)
    # mmdet reports 39.27 G for the 80-class model; 1 class: 38.94 GMAC = 77.9 GFLOP
    assert abs(spec.macs - 38.94e9) < 0.02e9
    assert spec.n_priors == 8400 and spec.level_off == [0, 6400, 8000, 8400]


@pytest.mark.parametrize("size", [128, 160])
def test_spec_wiring_matches_oracle(sd, size):
    """Unrounded weights: the op list is the restated network up to fp32 summation order."""
    m = R.build_model(sd)
    spec, _ = D.build_rtmdet_m(sd, size, keep_f32=True)
    # frames twice the network size: the 2x area downscale of the bench's 720p frames, the
    # input statistics the seeded weights are calibrated for
    frame = np.random.default_rng(size).integers(0, 256, (size * 9 // 8, 2 * size, 3), dtype=np.uint8)
    img, _, _ = R.letterbox(frame, size)
    x = R.normalize(img)
    with torch.no_grad():
        cs, bp = m(x)
        sc, bx = R.candidates(cs, bp, size)
        logits = torch.cat([c[0, 0].reshape(-1) for c in cs])
        x4 = torch.zeros((1, size, size, 4))
        x4[..., :3] = x[0].permute(1, 2, 0)
        cand = det_interp.run_spec(spec, x4)
    assert torch.allclose(cand[0, :, 5], logits, rtol=1e-4, atol=1e-3)
    assert torch.allclose(cand[0, :, 1:5], bx, rtol=1e-4, atol=2e-2)


def test_spec_bf16_weights_close_to_oracle(sd):
    """The device's bf16 weights alone move the logits by O(0.1) on these seeded weights."""
    size = 128
    m = R.build_model(sd)
    spec, _ = D.build_rtmdet_m(sd, size)
    frame = np.random.default_rng(7).integers(0, 256, (144, 256, 3), dtype=np.uint8)
    x = R.normalize(R.letterbox(frame, size)[0])
    with torch.no_grad():
        cs, _ = m(x)
        logits = torch.cat([c[0, 0].reshape(-1) for c in cs])
        x4 = torch.zeros((1, size, size, 4))
        x4[..., :3] = x[0].permute(1, 2, 0)
        cand = det_interp.run_spec(spec, x4)
    d = (cand[0, :, 5] - logits).abs() / (1 + logits.abs())
    assert float(d.max()) < 0.1 and float(d.mean()) < 0.02


def test_resize_area_fast_path():
    img = np.random.default_rng(0).integers(0, 256, (72, 128, 3), dtype=np.uint8)
    r = R.opencv_resize_linear_u8(img, 36, 64)
    a = img.astype(np.int32)
    exp = (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
    assert np.array_equal(r, exp.astype(np.uint8))


def test_resize_bilinear_properties():
    rng = np.random.default_rng(1)
    const = np.full((90, 160, 3), 77, np.uint8)
    assert (R.opencv_resize_linear_u8(const, 30, 53) == 77).all()  # 1/3 scale: fixed-point weights sum to 2048
    img = rng.integers(0, 256, (50, 70, 3), dtype=np.uint8)
    assert np.array_equal(R.opencv_resize_linear_u8(img, 50, 70), img)  # identity scale
    up = R.opencv_resize_linear_u8(img, 100, 140).astype(int)  # 2x upscale stays within the source range
    assert up.min() >= img.min() and up.max() <= img.max()


def test_letterbox_geometry():
    f = np.zeros((1080, 1920, 3), np.uint8)
    img, sf, (nh, nw) = R.letterbox(f, 640)
    assert (nh, nw) == (360, 640) and sf == (640 / 1920, 360 / 1080)
    assert (img[360:] == 114).all() and (img[:360] == 0).all()
    assert D.rescale_size(720, 1280) == (360, 640) and D.rescale_size(300, 500) == (384, 640)


def test_nms_restatement():
    boxes = torch.tensor([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [0, 0, 10, 10.5]], dtype=torch.float32)
    scores = torch.tensor([0.9, 0.8, 0.7, 0.9])
    keep = R.nms(boxes, scores, 0.6)
    # equal scores: the lower index first (stable); box 3 overlaps box 0 (IoU 0.95), box 1 (0.68)
    assert keep.tolist() == [0, 2]


def test_postprocess_candidates_first_is_argmax():
    """After NMS the first detection is the best-scoring valid prior: the GPU's per-frame
    argmax (mvp_det_forward's best row) is the reference's selected box."""
    rng = np.random.default_rng(3)
    P = 300
    sc = torch.tensor(rng.uniform(0, 0.6, P), dtype=torch.float32)
    xy = rng.uniform(0, 500, (P, 2))
    wh = rng.uniform(1, 100, (P, 2))
    bx = torch.tensor(np.concatenate([xy, xy + wh], 1), dtype=torch.float32)
    b, s, l = R.postprocess_candidates(sc, bx, [0, 200, 280, 300], (0.5, 0.5))
    i = int(torch.argmax(sc))
    assert torch.equal(b[0], bx[i] * 2) and float(s[0]) == float(sc[i])
    assert len(s) <= 100 and bool((s[:-1] >= s[1:]).all())


def _create(spec, ops=None, size=None, n_priors=None, w_elems=None):
    """mvp_det_create on dummy (never dereferenced) weight pointers: the graph is validated
    before any HIP call, so argument errors surface here on the CPU."""
    import ctypes
    from mvpose import _lib
    from mvpose.hrnet import TensorDesc
    ops = list(spec.ops) if ops is None else ops
    tens = (TensorDesc * len(spec.tensors))(*[TensorDesc(*t) for t in spec.tensors])
    arr = (D.DetOp * len(ops))(*ops)
    w, f = spec.blobs()
    h = ctypes.c_void_p()
    return _lib.lib.mvp_det_create(tens, len(spec.tensors), arr, len(ops), 0, size or spec.size,
                                   n_priors if n_priors is not None else spec.n_priors, ctypes.c_void_p(16),
                                   w.size if w_elems is None else w_elems, ctypes.c_void_p(16), f.size, 4,
                                   ctypes.byref(h)), h


def test_det_create_rejects_malformed_graphs(sd):
    import copy
    from mvpose import _lib
    spec, _ = D.build_rtmdet_m(sd, 128)
    k = next(i for i, op in enumerate(spec.ops) if op.kind == D.DET_CONV and op.ks == 3 and op.in_.c >= 64)
    bad = copy.deepcopy(list(spec.ops))
    bad[k].in_.c = 48  # a valid view, but cin not a multiple of 32
    rc, _ = _create(spec, bad)
    assert rc == -1 and "multiple of 32" in _lib.last_error()
    bad = copy.deepcopy(list(spec.ops))
    bad[k].out = bad[k].in_  # a conv writing its own input tensor
    rc, _ = _create(spec, bad)
    assert rc == -1
    rc, _ = _create(spec, n_priors=spec.n_priors + 1)  # head rows do not cover n_priors
    assert rc == -1 and "priors" in _lib.last_error()
    rc, _ = _create(spec, w_elems=1000)  # weights outside the blob
    assert rc == -1 and "blob" in _lib.last_error()
    rc, _ = _create(spec, size=100)
    assert rc == -1 and "multiple of 32" in _lib.last_error()
    bad = copy.deepcopy(list(spec.ops))
    bad[0].kind = 42
    rc, _ = _create(spec, bad)
    assert rc == -1 and "unknown kind" in _lib.last_error()


def test_det_nms_rejects_bad_levels():
    import ctypes
    from mvpose import _lib
    offs = (ctypes.c_int * 4)(0, 6400, 8000, 8400)
    # level offsets must start at 0 and end at n_priors; nms_pre <= 1024
    assert _lib.lib.mvp_det_nms(None, 1, 8000, offs, 3, 1000, 0.05, 0.6, 100, 2.0, 2.0, None, None, None) == -1
    assert _lib.lib.mvp_det_nms(None, 1, 8400, offs, 3, 2000, 0.05, 0.6, 100, 2.0, 2.0, None, None, None) == -1
    big = (ctypes.c_int * 2)(0, 9000)
    assert _lib.lib.mvp_det_nms(None, 1, 9000, big, 1, 1000, 0.05, 0.6, 100, 2.0, 2.0, None, None, None) == -1
    assert _lib.lib.mvp_det_nms(None, 0, 8400, offs, 3, 1000, 0.05, 0.6, 100, 2.0, 2.0, None, None, None) == 0
