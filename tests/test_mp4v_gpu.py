"""GPU: the split MPEG-4 Part 2 decode — host entropy decoding (mvp_mp4v_parse) + device
reconstruction (mvp_mp4v_reconstruct, csrc/mp4v_recon.hip) — returns, on the device, exactly the
BGR frames the host decoder (mvp_mp4v_decode) writes: every frame, every slice, every container
(MP4 / AVI / raw), mixed macroblock types (1MV, 4MV, skip, intra-in-P), a not-coded VOP, sizes
that are not multiples of 16 with vectors past the picture edge, MPEG quantisation, GOPs of
different lengths decoded as parallel slots.  Replaces cv.VideoCapture's decode of the
reference's mp4v recordings (utils.py:849-909; synchronize_videos.py:64,240); parity against
cv2 / FFmpeg is unpinned (neither exists in this image)."""
import numpy as np
import pytest
import torch

import mp4v_writer as W
from test_mp4v_split import mixed_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def video():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import video as v
    return v


def _gops(n_gops, w_mb, h_mb, seed, vol=None, qt=0):
    """n_gops GOPs of different lengths (mixed_stream: I + P + not-coded + P ...) back to back."""
    cfg, samples = None, []
    for g in range(n_gops):
        c, s, w, h = mixed_stream(w_mb, h_mb, 1 + (g % 3), seed + g, vol_wh=vol, quant_type=qt)
        cfg = c
        samples += s
    return cfg, samples, w, h


@pytest.mark.parametrize("w_mb,h_mb,vol,qt", [(4, 3, None, 0), (5, 3, (72, 40), 0), (4, 3, None, 1),
                                              (3, 2, (41, 19), 0)])
def test_device_frames_equal_host_frames(video, w_mb, h_mb, vol, qt):
    cfg, samples, w, h = _gops(5, w_mb, h_mb, 10 * w_mb + h_mb, vol, qt)
    host = video.decode_mp4v(cfg, samples, 0, None, threads=1)
    for sl in [(0, None), (0, -1), (3, 11), (7, 8), (len(samples) - 1, None)]:
        got = video.decode_mp4v_device(cfg, samples, *sl, threads=4)
        torch.cuda.synchronize()
        assert got.is_cuda and got.dtype == torch.uint8 and got.shape[1:] == (h, w, 3)
        np.testing.assert_array_equal(got.cpu().numpy(), host[slice(*sl)], err_msg=f"slice {sl}")


def test_device_decode_720p_stream(video):
    """The bench's 1280x720 mp4v workload shape (I + 11 P, +-3 px motion): 2 GOPs, bit-identical."""
    rng = np.random.default_rng(3)
    w, h = 1280, 720
    mw, mh = w // 16, h // 16

    def intra():
        b = np.zeros((6, 64), np.int64)
        for n in range(6):
            b[n, 0] = rng.integers(40, 160) if n < 4 else rng.integers(80, 140)
            m = rng.random(63) < 0.05
            b[n, 1:][m] = rng.integers(-4, 5, m.sum())
        return {"q": 6, "blocks": b, "ac_pred": False}

    def inter():
        b = np.zeros((6, 64), np.int64)
        m = rng.random((6, 64)) < 0.01
        b[m] = rng.integers(-2, 3, m.sum())
        return {"type": "inter", "mv": (int(rng.integers(-6, 7)), int(rng.integers(-6, 7))), "blocks": b}

    vw = W.VopWriter(w, h)
    i_vop = vw.i_vop([[intra() for _ in range(mw)] for _ in range(mh)], 6)
    p_vops = [vw.p_vop([[inter() for _ in range(mw)] for _ in range(mh)], 6, rounding=k % 2) for k in range(2)]
    samples = ([i_vop] + [p_vops[k % 2] for k in range(11)]) * 2
    cfg = W.vol_header(w, h)
    host = video.decode_mp4v(cfg, samples)
    got = video.decode_mp4v_device(cfg, samples).cpu().numpy()
    np.testing.assert_array_equal(got, host)


def test_read_recording_device_containers(video, tmp_path):
    """MP4, AVI (XVID) and raw .m4v containers through read_recording(device=...): the host
    reader's frames, on the device; the reference's [0, -1] slice drops the last frame."""
    from test_mp4v import _write_avi_mp4v
    cfg, samples, w, h = _gops(3, 4, 3, 77)
    host = video.decode_mp4v(cfg, samples)
    mp4 = tmp_path / "cam0_synced.mp4"
    mp4.write_bytes(W.mp4_file(cfg, samples, w, h, chunk=2))
    m4v = tmp_path / "cam0.m4v"
    m4v.write_bytes(cfg + b"".join(samples))
    avi = tmp_path / "cam0.avi"
    _write_avi_mp4v(avi, [cfg + samples[0]] + samples[1:], w, h)
    for p in (mp4, m4v, avi):
        got = video.read_recording(p, 0, -1, device="cuda")
        assert isinstance(got, torch.Tensor) and got.is_cuda
        np.testing.assert_array_equal(got.cpu().numpy(), host[:-1], err_msg=str(p))
