"""CPU: the native MPEG-4 Part 2 ('mp4v') decoder (csrc/mp4v.cpp, host code in libmvpose.so) that
replaces cv.VideoCapture on the reference's recordings (utils.py:849-909; the files
synchronize_videos.py:64,240 writes with cv2.VideoWriter_fourcc(*'mp4v')).

Parity against cv2 / FFmpeg is UNPINNED: neither exists in this image and the reference holds no
video fixture.  What is pinned: bitstreams written from known quantised coefficients and motion
vectors (tests/mp4v_writer.py, a separate transcription of the standard's VLC tables and
prediction rules) decode to exactly the frames a numpy restatement of inverse quantisation,
FFmpeg's simple IDCT and half-pel motion compensation reconstructs from those values; the
restated IDCT meets the IEEE 1180 accuracy limits against the float IDCT; the decoder's tables
pass their structural self-check; MP4, AVI and raw elementary-stream containers give the same
frames."""
import os

import numpy as np
import pytest

import mp4v_writer as W
from mvpose import _lib, video

WH = (64, 48)


def _decode_yuv(config, samples):
    dec = video.Mp4vDecoder(config)
    try:
        return [dec.decode(s, yuv=True) for s in samples]
    finally:
        dec.close()


def _planes(buf, w, h):
    y = buf[:w * h].reshape(h, w)
    u = buf[w * h:w * h + (w // 2) * (h // 2)].reshape(h // 2, w // 2)
    v = buf[w * h + (w // 2) * (h // 2):].reshape(h // 2, w // 2)
    return [y, u, v]


def _rand_intra_mb(rng, q, ac_pred=False, density=0.15, amp=6):
    blocks = np.zeros((6, 64), np.int64)
    for n in range(6):
        blocks[n, 0] = rng.integers(40, 160) if n < 4 else rng.integers(80, 140)
        m = rng.random(63) < density
        blocks[n, 1:][m] = rng.integers(-amp, amp + 1, m.sum())
    return {"q": q, "blocks": blocks, "ac_pred": ac_pred}


def _rand_residual(rng, density=0.08, amp=4):
    blocks = np.zeros((6, 64), np.int64)
    m = rng.random((6, 64)) < density
    blocks[m] = rng.integers(-amp, amp + 1, m.sum())
    return blocks


def test_decoder_tables_selfcheck():
    _lib.call("mvp_mp4v_selfcheck")


def test_writer_tables_are_the_standards_lmax_rmax():
    """The writer's TCOEF transcription reproduces the standard's LMAX / RMAX tables (escape
    types 1 / 2), a third, independent check on the run / level layout."""
    lmax_intra0 = [27, 10, 5, 4, 3, 3, 3, 3, 2, 2, 1, 1, 1, 1, 1]
    lmax_intra1 = [8, 3, 2, 2, 2, 2, 2] + [1] * 14
    lmax_inter0 = [12, 6, 4, 3, 3, 3, 3, 2, 2, 2, 2] + [1] * 16
    lmax_inter1 = [3, 2] + [1] * 39
    for intra, last, ref in ((True, 0, lmax_intra0), (True, 1, lmax_intra1), (False, 0, lmax_inter0),
                             (False, 1, lmax_inter1)):
        assert [W.LMAX[intra][(last, r)] for r in range(len(ref))] == ref
        assert (last, len(ref)) not in W.LMAX[intra]
    assert [W.RMAX[True][(0, lv)] for lv in (1, 2, 3, 4, 5, 6, 11)] == [14, 9, 7, 3, 2, 1, 0]
    assert [W.RMAX[False][(0, lv)] for lv in (1, 2, 3, 4, 5, 7)] == [26, 10, 6, 2, 1, 0]
    assert [W.RMAX[False][(1, lv)] for lv in (1, 2, 3)] == [40, 1, 0]
    codes = sorted(W.TCOEF[True].values()) + [W.ESCAPE]
    assert sorted(codes) == sorted(list(W.TCOEF[False].values()) + [W.ESCAPE])
    bits = [format(c, f"0{n}b") for c, n in codes]
    assert not any(a != b and b.startswith(a) for a in bits for b in bits)
    assert sorted(W.ALT_V) == list(range(64)) and sorted(W.ALT_H) == list(range(64))


def test_simple_idct_meets_ieee1180():
    """The restated simple IDCT against the float IDCT on IEEE 1180-style random blocks
    (coefficients of the forward DCT of random pixels in [-L, H]): peak error <= 1, per-pixel
    mean square error <= 0.06, overall mean error <= 0.0015."""
    rng = np.random.default_rng(1180)
    k = np.arange(8)
    cu = np.where(k == 0, np.sqrt(0.125), 0.5)
    basis = cu[:, None] * np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16)
    for lo, hi in ((-256, 255), (-5, 5)):
        err = []
        for _ in range(2000):
            px = rng.integers(lo, hi + 1, (8, 8)).astype(np.float64)
            coef = np.clip(np.round(basis @ px @ basis.T), -2048, 2047)
            ref = np.clip(np.round(W.float_idct(coef)), -256, 255)
            got = np.clip(W.simple_idct(coef), -256, 255)
            err.append(got - ref)
        e = np.array(err)
        assert np.abs(e).max() <= 1
        assert (e ** 2).mean(0).max() <= 0.06
        assert abs(e.mean()) <= 0.0015


@pytest.mark.parametrize("ac_pred", [False, True])
def test_intra_vop_known_coefficients(ac_pred):
    """An I-VOP of known quantised coefficients, per-MB DQUANT, DC prediction everywhere (and AC
    prediction with QP rescaling) decodes to the restated reconstruction bit for bit."""
    w, h = WH
    rng = np.random.default_rng(7 + ac_pred)
    qs = np.clip(8 + np.cumsum(rng.integers(-2, 3, w // 16 * h // 16)), 2, 31).reshape(h // 16, w // 16)
    mbs = [[_rand_intra_mb(rng, int(qs[y, x]), ac_pred=ac_pred and (x + y) % 2 == 0) for x in range(w // 16)]
           for y in range(h // 16)]
    vw = W.VopWriter(w, h)
    cfg = W.vol_header(w, h)
    vop = vw.i_vop(mbs, int(qs[0, 0]))
    got = _planes(_decode_yuv(cfg, [vop])[0], w, h)
    exp = W.reconstruct(w, h, [("I", mbs, int(qs[0, 0]), 0)])[0]
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)


def test_escape_codes():
    """Levels past LMAX (escape 1), runs past RMAX (escape 2) and fixed-length events (escape 3)."""
    w, h = 32, 16
    blocks = np.zeros((6, 64), np.int64)
    blocks[:, 0] = 100
    blocks[0, 1] = 40          # run 0, level 40 > 27: escape 1 (27 + 13) or 3
    blocks[0, W.ZIGZAG[12]] = 3  # long-ish run, level 3
    blocks[1, W.ZIGZAG[40]] = 1  # run 38 at level 1 (intra RMAX 14): escape 2 / 3
    blocks[2, W.ZIGZAG[5]] = -300  # escape 3
    blocks[3, W.ZIGZAG[63]] = 2
    mbs = [[{"q": 4, "blocks": blocks, "ac_pred": False}, _rand_intra_mb(np.random.default_rng(3), 4)]]
    vw = W.VopWriter(w, h)
    cfg = W.vol_header(w, h)
    vop = vw.i_vop(mbs, 4)
    got = _planes(_decode_yuv(cfg, [vop])[0], w, h)
    exp = W.reconstruct(w, h, [("I", mbs, 4, 0)])[0]
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)


@pytest.mark.parametrize("rounding,fcode", [(0, 1), (1, 1), (0, 2), (1, 3)])
def test_p_vop_known_motion(rounding, fcode):
    """I-VOP then P-VOPs mixing not-coded, 1MV (full / half-pel, pointing outside the frame),
    4MV, intra and DQUANT macroblocks with residuals: the restated half-pel prediction (rounding
    control, edge clamping, 1MV / 4MV chroma vectors) + residual, bit for bit."""
    w, h = 80, 48
    mw, mh = w // 16, h // 16
    rng = np.random.default_rng(100 + 10 * rounding + fcode)
    lim = (32 << (fcode - 1)) - 1
    iv = [[_rand_intra_mb(rng, 6) for _ in range(mw)] for _ in range(mh)]
    vops = [("I", iv, 6, 0)]
    vw = W.VopWriter(w, h)
    cfg = W.vol_header(w, h)
    samples = [vw.i_vop(iv, 6)]
    for f in range(3):
        mbs, q = [], 6
        for y in range(mh):
            row = []
            for x in range(mw):
                k = (x + 2 * y + f) % 6
                if k == 0:
                    mb = {"type": "skip"}
                elif k == 1:
                    mb = {"type": "inter", "mv": (int(rng.integers(-lim, lim + 1)), int(rng.integers(-lim, lim + 1))),
                          "blocks": _rand_residual(rng)}
                elif k == 2:
                    mb = {"type": "inter4v", "mvs": [(int(rng.integers(-9, 10)), int(rng.integers(-9, 10)))
                                                     for _ in range(4)], "blocks": _rand_residual(rng)}
                elif k == 3:
                    mb = dict(_rand_intra_mb(rng, q), type="intra")
                elif k == 4:
                    q = int(np.clip(q + rng.integers(-2, 3), 2, 31))
                    mb = {"type": "inter", "mv": (int(rng.integers(-5, 6)), int(rng.integers(-5, 6))), "q": q,
                          "blocks": _rand_residual(rng)}
                else:
                    mb = {"type": "inter", "mv": (0, 0), "blocks": np.zeros((6, 64))}
                if mb["type"] not in ("skip", "inter4v"):
                    mb.setdefault("q", q)
                q = mb.get("q", q)
                row.append(mb)
            mbs.append(row)
        samples.append(vw.p_vop(mbs, 6, rounding=rounding, fcode=fcode))
        vops.append(("P", mbs, 6, rounding))
    got = [_planes(b, w, h) for b in _decode_yuv(cfg, samples)]
    exp = W.reconstruct(w, h, vops, fcode)
    for f, (gf, ef) in enumerate(zip(got, exp)):
        for p, (g, e) in enumerate(zip(gf, ef)):
            np.testing.assert_array_equal(g, e, err_msg=f"frame {f} plane {p}")


def _stream(n_p=4, seed=5):
    w, h = WH
    rng = np.random.default_rng(seed)
    mw, mh = w // 16, h // 16
    vw = W.VopWriter(w, h)
    samples = [vw.i_vop([[_rand_intra_mb(rng, 5) for _ in range(mw)] for _ in range(mh)], 5)]
    for f in range(n_p):
        mbs = [[{"type": "inter", "mv": (int(rng.integers(-6, 7)), int(rng.integers(-6, 7))),
                 "blocks": _rand_residual(rng)} for _ in range(mw)] for _ in range(mh)]
        samples.append(vw.p_vop(mbs, 5, rounding=f % 2))
    return W.vol_header(w, h), samples


def test_containers_give_the_same_frames(tmp_path):
    """The same stream as an MP4 (esds config, stsc / stco / stsz sample tables), an AVI with the
    XVID FourCC (VOL headers in the first chunk) and a raw .m4v elementary stream: identical BGR
    frames, sliced [start:end] with Python semantics like the reference (read_recording)."""
    cfg, samples = _stream()
    w, h = WH
    dec = video.Mp4vDecoder(cfg)
    ref = np.stack([dec.decode(s) for s in samples])
    dec.close()
    assert ref.shape == (5, h, w, 3) and ref.dtype == np.uint8
    mp4 = tmp_path / "cam0_synced.mp4"
    mp4.write_bytes(W.mp4_file(cfg, samples, w, h, chunk=2))
    np.testing.assert_array_equal(video.read_recording(mp4, 0, None), ref)
    np.testing.assert_array_equal(video.read_recording(mp4), ref[0:-1])        # the reference's [0, -1]
    np.testing.assert_array_equal(video.read_recording(mp4, 2, 4), ref[2:4])
    info = video.parse_mp4(mp4.read_bytes())
    assert (info.width, info.height, len(info)) == (w, h, 5) and abs(info.fps - 30) < 1e-9
    m4v = tmp_path / "cam0.m4v"
    m4v.write_bytes(cfg + b"".join(samples))
    np.testing.assert_array_equal(video.read_recording(m4v, 0, None), ref)
    avi = tmp_path / "cam0.avi"
    _write_avi_mp4v(avi, [cfg + samples[0]] + samples[1:], w, h)
    np.testing.assert_array_equal(video.read_recording(avi, 0, None), ref)


def _write_avi_mp4v(path, chunks, w, h):
    import struct

    def chunk(cc4, data):
        return cc4 + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")

    def lst(kind, body):
        return b"LIST" + struct.pack("<I", len(body) + 4) + kind + body

    avih = struct.pack("<IIIIIIIIII16x", 33333, 0, 0, 0x10, len(chunks), 0, 1, 0, w, h)
    strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", b"XVID", 0, 0, 0, 0, 1000, 30000, 0, len(chunks), 0,
                       0xFFFFFFFF, 0, 0, 0, w, h)
    strf = struct.pack("<IiiHHIIiiII", 40, w, h, 1, 12, struct.unpack("<I", b"XVID")[0], w * h * 3 // 2, 0, 0, 0, 0)
    hdrl = lst(b"hdrl", chunk(b"avih", avih) + lst(b"strl", chunk(b"strh", strh) + chunk(b"strf", strf)))
    movi = lst(b"movi", b"".join(chunk(b"00dc", c) for c in chunks))
    body = b"AVI " + hdrl + movi
    path.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_not_coded_vop_repeats_the_frame():
    cfg, samples = _stream(n_p=1)
    w, h = WH
    tb = W.time_bits(30)
    bw = W.BitWriter()
    bw.start_code(0xB6)
    bw.put(1, 2)
    bw.put(0, 1)
    bw.put(1, 1)
    bw.put(3, tb)
    bw.put(1, 1)
    bw.put(0, 1)              # vop_coded = 0
    bw.stuff()
    dec = video.Mp4vDecoder(cfg)
    a = [dec.decode(s) for s in samples]
    b = dec.decode(bw.tobytes())
    dec.close()
    np.testing.assert_array_equal(a[-1], b)


def test_unsupported_streams_raise():
    cfg, samples = _stream(n_p=0)
    bw = W.BitWriter()
    bw.start_code(0xB6)
    bw.put(2, 2)              # B-VOP
    bw.put(0, 1)
    bw.put(1, 1)
    bw.put(0, W.time_bits(30))
    bw.put(1, 1)
    bw.put(1, 1)
    bw.stuff()
    dec = video.Mp4vDecoder(cfg)
    dec.decode(samples[0])
    with pytest.raises(_lib.MvposeError, match="B-VOPs"):
        dec.decode(bw.tobytes())
    dec.close()
    with pytest.raises(_lib.MvposeError, match="no video object layer"):
        video.Mp4vDecoder(b"\0\0\1\xb0\x01")
    # an H.264 MP4 names its codec instead of decoding garbage
    raw = bytearray(W.mp4_file(cfg, samples, *WH))
    i = raw.index(b"mp4v")
    raw[i:i + 4] = b"avc1"
    with pytest.raises(NotImplementedError, match="avc1"):
        video.parse_mp4(bytes(raw))


def test_bgr_conversion_is_bt601_limited_range():
    """Flat grey / saturated patches through the I420 -> BGR conversion (BT.601, limited range;
    cv2's swscale rounding is unpinned): Y = 16 / 235 with neutral chroma give 0 / 255."""
    w, h = 32, 16
    mbs = [[{"q": 2, "blocks": np.zeros((6, 64)) + np.array([[v] + [0] * 63] * 4 + [[128] + [0] * 63] * 2),
             "ac_pred": False} for v in (16, 235)]]
    # DC level v at QP 2 (dc_scale 8): pixel value v * 8 / 8 = v
    vw = W.VopWriter(w, h)
    dec = video.Mp4vDecoder(W.vol_header(w, h))
    bgr = dec.decode(vw.i_vop(mbs, 2))
    dec.close()
    assert (bgr[:, :16] == 0).all() and (bgr[:, 16:] == 255).all()


def test_parallel_gop_decode_equals_serial():
    """decode_mp4v splits the stream at I-VOPs and decodes the GOPs holding wanted frames on a
    thread pool: the same frames as one decoder walking every sample, for every slice."""
    w, h = WH
    rng = np.random.default_rng(11)
    mw, mh = w // 16, h // 16
    vw = W.VopWriter(w, h)
    samples = []
    for n_p in (2, 3, 1, 0, 2):
        samples.append(vw.i_vop([[_rand_intra_mb(rng, 4) for _ in range(mw)] for _ in range(mh)], 4))
        for f in range(n_p):
            mbs = [[{"type": "inter", "mv": (int(rng.integers(-5, 6)), int(rng.integers(-5, 6))),
                     "blocks": _rand_residual(rng)} for _ in range(mw)] for _ in range(mh)]
            samples.append(vw.p_vop(mbs, 4, rounding=f % 2))
    cfg = W.vol_header(w, h)
    assert [video.vop_coding_type(s) for s in samples] == [0, 1, 1, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1]
    dec = video.Mp4vDecoder(cfg)
    serial = np.stack([dec.decode(s) for s in samples])
    dec.close()
    for sl in [(0, None), (0, -1), (2, 9), (4, 5), (8, None), (12, 13), (5, 3)]:
        for threads in (1, 4):
            got = video.decode_mp4v(cfg, samples, *sl, threads=threads)
            np.testing.assert_array_equal(got, serial[slice(*sl)], err_msg=f"{sl} threads={threads}")


def test_repeated_vol_keeps_the_reference_frame():
    """A VOL repeated in front of a P-VOP or a not-coded VOP (encoders without a global header
    repeat it) refreshes per-VOL state only: the P-VOP still predicts from the previous picture
    and a not-coded VOP still repeats it (alloc() used to reset both to grey)."""
    cfg, samples = _stream(n_p=3)
    dec = video.Mp4vDecoder(cfg)
    plain = [dec.decode(s).copy() for s in samples]
    dec.close()
    dec = video.Mp4vDecoder(cfg)
    again = [dec.decode(s if k == 0 else cfg + s).copy() for k, s in enumerate(samples)]
    dec.close()
    for k, (a, b) in enumerate(zip(plain, again)):
        np.testing.assert_array_equal(a, b, err_msg=f"frame {k}")


def test_vol_size_change_is_rejected():
    """A later VOL that changes the frame size inside one stream raises instead of writing the
    new size into buffers sized from the first VOL (heap overflow in host code)."""
    cfg, samples = _stream(n_p=1)
    w, h = WH
    dec = video.Mp4vDecoder(cfg)
    dec.decode(samples[0])
    with pytest.raises(_lib.MvposeError, match="changes the frame size"):
        dec.decode(W.vol_header(w + 16, h) + samples[1])
    with pytest.raises(ValueError, match="I420"):
        dec.decode(samples[1], yuv=True, out=np.empty(10, np.uint8))
    dec.close()
