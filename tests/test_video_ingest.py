"""Recording ingest (reference utils.py:849-909 frame_generator /
read_video_as_frames / process_image_files): MJPEG and uncompressed AVI, frame<N>.jpg
directories and .npy stacks -> (T, H, W, 3) uint8 BGR, sliced [start:end] with the
reference's [0, -1] default.  The reference ships no recordings, and cv2 (whose
VideoCapture decodes MJPEG with FFmpeg) is absent, so decoded MJPEG pixels are checked
against libjpeg decoding the same bitstreams (parity with cv2 unpinned); uncompressed
frames are bit-exact round trips."""
import io
import os
import struct

import numpy as np
import pytest

from mvpose import pose_estimation, video

PIL = pytest.importorskip("PIL.Image")


def _frames(T=5, H=24, W=37, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    base = np.stack([(x * 7 + y * 3) % 256, (x * 2 + y * 9) % 256, (x * y) % 256], -1)
    return np.stack([(base + t * 11 + rng.integers(0, 8, base.shape)) % 256 for t in range(T)]).astype(np.uint8)


def _jpeg_bgr(fr):
    """libjpeg's decode of PIL's encoding of one BGR frame (what write_avi stores)."""
    b = io.BytesIO()
    PIL.fromarray(np.ascontiguousarray(fr[:, :, ::-1])).save(b, "JPEG", quality=90)
    return np.asarray(PIL.open(io.BytesIO(b.getvalue())).convert("RGB"))[:, :, ::-1]


def test_uncompressed_avi_roundtrip_bit_exact(tmp_path):
    fr = _frames(W=37)                        # 111-byte rows: DIB stride padding
    p = str(tmp_path / "cam0.avi")
    video.write_avi(p, fr, codec="rgb")
    info = video.parse_avi(open(p, "rb").read())
    assert (info.width, info.height, info.codec, len(info)) == (37, 24, "rgb", 5)
    np.testing.assert_array_equal(video.read_avi(p), fr)
    np.testing.assert_array_equal(video.read_recording(p), fr[:-1])      # [0, -1]: last frame dropped
    np.testing.assert_array_equal(video.read_recording(p, 1, 3), fr[1:3])


def test_mjpeg_avi_matches_libjpeg(tmp_path):
    y, x = np.mgrid[0:32, 0:48]
    fr = np.stack([np.stack([128 + 60 * np.sin((x + t) / 5), 128 + 50 * np.cos(y / 7), 100 + x + y], -1)
                   for t in range(6)]).astype(np.uint8)      # smooth: JPEG q90 stays close
    p = str(tmp_path / "cam1.avi")
    video.write_avi(p, fr, fps=25.0, codec="mjpeg")
    info = video.parse_avi(open(p, "rb").read())
    assert info.codec == "mjpeg" and abs(info.fps - 25.0) < 1e-9
    got = video.read_avi(p)
    want = np.stack([_jpeg_bgr(f) for f in fr])
    np.testing.assert_array_equal(got, want)
    err = np.abs(got.astype(int) - fr.astype(int)).mean()
    assert err < 3, err                        # and it is a picture of the input (q90)


def test_avi_junk_rec_lists_and_truncation(tmp_path):
    """Chunks the walker must step over (JUNK, odd sizes, 'rec ' groups, ix00 indexes) and a
    recording cut mid-frame: the complete frames are returned."""
    fr = _frames(T=4, H=8, W=6, seed=2)
    stride = 20                                # 18 bytes of pixels padded to 4
    def ck(cc, data):
        return cc + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")
    def ls(kind, body):
        return b"LIST" + struct.pack("<I", len(body) + 4) + kind + body
    strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", b"\0\0\0\0", 0, 0, 0, 0, 1, 30, 0, 4, 0, 0, 0, 0, 0, 6, 8)
    strf = struct.pack("<IiiHHIIiiII", 40, 6, -8, 1, 24, 0, stride * 8, 0, 0, 0, 0)   # top-down rows
    hdrl = ls(b"hdrl", ck(b"avih", b"\0" * 56) + ls(b"strl", ck(b"strh", strh) + ck(b"strf", strf)))
    frames = []
    for f in fr:
        rows = np.zeros((8, stride), np.uint8)
        rows[:, :18] = f.reshape(8, 18)
        frames.append(ck(b"00db", rows.tobytes()))
    movi = ls(b"movi", ck(b"JUNK", b"abc") + ls(b"rec ", frames[0] + frames[1]) + ck(b"ix00", b"\0" * 8) +
              frames[2] + ck(b"01wb", b"audio") + frames[3])
    body = b"AVI " + ck(b"JUNK", b"x" * 5) + hdrl + movi
    blob = b"RIFF" + struct.pack("<I", len(body)) + body
    p = tmp_path / "odd.avi"
    p.write_bytes(blob)
    np.testing.assert_array_equal(video.read_avi(str(p)), fr)
    p.write_bytes(blob[:-30])                  # the last frame is cut
    np.testing.assert_array_equal(video.read_avi(str(p)), fr[:3])


def test_image_directory_numeric_order(tmp_path):
    fr = _frames(T=3, H=16, W=16, seed=3)
    for n, f in zip((2, 10, 1), fr):           # frame10 sorts after frame2 (integer key, utils.py:853-856)
        PIL.fromarray(np.ascontiguousarray(f[:, :, ::-1])).save(tmp_path / f"frame{n}.jpg", quality=90)
    (tmp_path / "notes.txt").write_text("ignored")
    got = video.read_recording(str(tmp_path), 0, None)
    want = np.stack([_jpeg_bgr(fr[2]), _jpeg_bgr(fr[0]), _jpeg_bgr(fr[1])])
    np.testing.assert_array_equal(got, want)


def test_load_frames_dispatch_and_errors(tmp_path):
    fr = _frames(T=4)
    a = str(tmp_path / "a.avi")
    video.write_avi(a, fr, codec="rgb")
    n = str(tmp_path / "b.npy")
    np.save(n, fr)
    out = pose_estimation.load_frames([a, n], (1, -1))
    np.testing.assert_array_equal(out[0], fr[1:-1])
    np.testing.assert_array_equal(out[1], fr[1:-1])
    assert pose_estimation.load_frames("not-a-list") is None
    m = tmp_path / "c.mp4"
    m.write_bytes(b"\0\0\0\x18ftypmp42" + b"\0" * 32)
    with pytest.raises(ValueError):          # an MP4 without its moov box
        pose_estimation.load_frames([str(m)])
    k = tmp_path / "d.mkv"
    k.write_bytes(b"\x1a\x45\xdf\xa3" + b"\0" * 32)   # Matroska: no demuxer here
    with pytest.raises(NotImplementedError):
        pose_estimation.load_frames([str(k)])
    with pytest.raises(FileNotFoundError):
        pose_estimation.load_frames([str(tmp_path / "missing.avi")])
    with pytest.raises(ValueError):
        video.parse_avi(b"RIFF\0\0\0\0WAVE")
