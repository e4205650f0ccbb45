"""CPU: the host half of the split MPEG-4 Part 2 decode (mvp_mp4v_parse, csrc/mp4v.cpp parse mode)
— one 32-B record per macroblock + the inverse-quantised coefficients — carries everything the
picture needs: a numpy restatement of the device reconstruction (csrc/mp4v_recon.hip: FFmpeg's
simple IDCT from tests/mp4v_writer.py, half-pel prediction with per-pixel edge clamping, the
host decoder's buffer swap) rebuilds, from the records alone, exactly the I420 pictures the
host decoder (mvp_mp4v_decode) outputs.  Streams: I + 1MV P-VOPs, 4MV / skip / intra-in-P
macroblocks, a not-coded VOP, frame sizes that are not multiples of 16 (vectors pointing past
the visible edge), MPEG quantisation.  tests/test_mp4v_gpu.py holds the device kernel to the
host frames; the reference's own decoder (cv2 / FFmpeg) is absent: parity vs it is unpinned."""
import numpy as np
import pytest

import mp4v_writer as W
from mvpose import _lib, video

REC = np.dtype([("kind", "u1"), ("nnz", "u1", 6), ("pad", "u1"), ("mv", "<i2", (4, 2)), ("cmv", "<i2", 2),
                ("coef", "<u4")])
assert REC.itemsize == video.MB_REC_BYTES


def _mc(ref, vw, vh, x, y, mvx, mvy, rnd):
    """8x8 half-pel prediction at (x, y), coordinates clamped to the visible vw x vh picture."""
    sx, sy = x + (mvx >> 1), y + (mvy >> 1)
    xs = np.clip(np.arange(sx, sx + 9), 0, vw - 1)
    ys = np.clip(np.arange(sy, sy + 9), 0, vh - 1)
    p = ref[np.ix_(ys, xs)].astype(np.int64)
    a, b, c, d = p[:-1, :-1], p[:-1, 1:], p[1:, :-1], p[1:, 1:]
    hx, hy = mvx & 1, mvy & 1
    if not hx and not hy:
        return a
    if hx and not hy:
        return (a + b + 1 - rnd) >> 1
    if hy and not hx:
        return (a + c + 1 - rnd) >> 1
    return (a + b + c + d + 2 - rnd) >> 2


def reconstruct_records(parsed, w, h):
    """The device kernel restated: parsed = [(records, coefficients, coded, rounding)] of one GOP
    -> the I420 pictures (visible size) after each sample."""
    mw, mh = (w + 15) // 16, (h + 15) // 16
    pics = [[np.full((16 * mh, 16 * mw), 128, np.int64)] + [np.full((8 * mh, 8 * mw), 128, np.int64)
                                                             for _ in range(2)] for _ in range(2)]
    vis = [(w, h), ((w + 1) >> 1, (h + 1) >> 1), ((w + 1) >> 1, (h + 1) >> 1)]
    cur_i, out = 0, []
    for rec, coef, coded, rnd in parsed:
        if coded == 1:
            cur_i ^= 1
            cur, ref = pics[cur_i], pics[cur_i ^ 1]
            R = rec.view(REC)
            for m in range(mw * mh):
                r = R[m]
                if r["kind"] == 3:
                    continue
                mx, my = m % mw, m // mw
                blk = np.zeros((6, 64), np.int64)
                o = int(r["coef"])
                for n in range(6):
                    for e in coef[o:o + int(r["nnz"][n])]:
                        blk[n, int(e) >> 16] = np.int16(np.uint16(int(e) & 0xFFFF))
                    o += int(r["nnz"][n])
                for n in range(6):
                    res = W.simple_idct(blk[n])
                    if n < 4:
                        pl, x, y, mv = 0, 16 * mx + 8 * (n & 1), 16 * my + 8 * (n >> 1), r["mv"][n]
                    else:
                        pl, x, y, mv = n - 3, 8 * mx, 8 * my, r["cmv"]
                    if r["kind"] == 0:
                        val = res
                    else:
                        mvx, mvy = (int(mv[0]), int(mv[1])) if r["kind"] == 1 else (0, 0)
                        val = _mc(ref[pl], *vis[pl], x, y, mvx, mvy, rnd) + res
                    cur[pl][y:y + 8, x:x + 8] = np.clip(val, 0, 255)
        c = pics[cur_i]
        out.append(np.concatenate([c[0][:h, :w].ravel(), c[1][:vis[1][1], :vis[1][0]].ravel(),
                                   c[2][:vis[2][1], :vis[2][0]].ravel()]).astype(np.uint8))
    return out


def _intra(rng, q=5, density=0.15, amp=6, ac_pred=False):
    b = np.zeros((6, 64), np.int64)
    for n in range(6):
        b[n, 0] = rng.integers(40, 160) if n < 4 else rng.integers(80, 140)
        m = rng.random(63) < density
        b[n, 1:][m] = rng.integers(-amp, amp + 1, m.sum())
    return {"q": q, "blocks": b, "ac_pred": ac_pred}


def _residual(rng, density=0.08, amp=4):
    b = np.zeros((6, 64), np.int64)
    m = rng.random((6, 64)) < density
    b[m] = rng.integers(-amp, amp + 1, m.sum())
    return b


def mixed_stream(w_mb, h_mb, n_p, seed, vol_wh=None, quant_type=0, mvmax=12):
    """I-VOP + P-VOPs whose macroblocks mix 1MV, 4MV, skip and intra (+ a not-coded VOP after
    the first P), vectors up to +-mvmax half-pels (past the picture edge)."""
    rng = np.random.default_rng(seed)
    w, h = 16 * w_mb, 16 * h_mb
    vw = W.VopWriter(w, h)
    samples = [vw.i_vop([[_intra(rng, ac_pred=bool(rng.integers(0, 2))) for _ in range(w_mb)] for _ in range(h_mb)], 5)]

    def mv():
        return int(rng.integers(-mvmax, mvmax + 1)), int(rng.integers(-mvmax, mvmax + 1))

    for f in range(n_p):
        mbs = []
        for _ in range(h_mb):
            row = []
            for _ in range(w_mb):
                t = rng.choice(["inter", "inter4v", "skip", "intra"], p=[0.5, 0.25, 0.15, 0.1])
                if t == "inter":
                    row.append({"type": "inter", "mv": mv(), "blocks": _residual(rng)})
                elif t == "inter4v":
                    row.append({"type": "inter4v", "mvs": [mv() for _ in range(4)], "blocks": _residual(rng)})
                elif t == "skip":
                    row.append({"type": "skip"})
                else:
                    row.append({"type": "intra", **_intra(rng)})
            mbs.append(row)
        samples.append(vw.p_vop(mbs, 5, rounding=f % 2))
        if f == 0:                                   # a not-coded VOP: the previous frame again
            bw = W.BitWriter()
            bw.start_code(0xB6)
            bw.put(1, 2)
            bw.put(0, 1)
            bw.put(1, 1)
            bw.put(2, W.time_bits(30))
            bw.put(1, 1)
            bw.put(0, 1)
            bw.stuff()
            samples.append(bw.tobytes())
    vw_, vh_ = vol_wh or (w, h)
    return W.vol_header(vw_, vh_, quant_type=quant_type), samples, vw_, vh_


def _host_yuv(cfg, samples):
    dec = video.Mp4vDecoder(cfg)
    try:
        return [dec.decode(s, yuv=True).copy() for s in samples]
    finally:
        dec.close()


def _parse(cfg, samples):
    ps = video.Mp4vParser(cfg)
    out = []
    try:
        for s in samples:
            rec, coef, coded, rnd = ps.parse(s)     # views of the parser's scratch: copy
            out.append((None if rec is None else rec.copy(), coef.copy(), coded, rnd))
        return out
    finally:
        ps.close()


@pytest.mark.parametrize("w_mb,h_mb,vol,qt,seed", [(4, 3, None, 0, 1), (5, 3, (72, 40), 0, 2), (4, 3, None, 1, 3),
                                                   (3, 2, (41, 19), 0, 4)])
def test_records_rebuild_the_host_pictures(w_mb, h_mb, vol, qt, seed):
    cfg, samples, w, h = mixed_stream(w_mb, h_mb, 3, seed, vol_wh=vol, quant_type=qt)
    parsed = _parse(cfg, samples)
    assert [p[2] for p in parsed] == [1, 1, 0, 1, 1]
    kinds = np.concatenate([p[0].view(REC)["kind"] for p in parsed if p[0] is not None])
    assert {0, 1, 2} <= set(kinds.tolist()), set(kinds.tolist())
    got = reconstruct_records(parsed, w, h)
    exp = _host_yuv(cfg, samples)
    for k, (g, e) in enumerate(zip(got, exp)):
        np.testing.assert_array_equal(g, e, err_msg=f"sample {k}")


def test_parse_and_decode_do_not_mix_on_one_handle():
    cfg, samples, _, _ = mixed_stream(2, 2, 1, 5)
    ps = video.Mp4vParser(cfg)
    ps.parse(samples[0])
    with pytest.raises(_lib.MvposeError, match="parses"):
        import ctypes
        out = np.empty((32, 32, 3), np.uint8)
        data = np.frombuffer(samples[1], np.uint8)
        n = ctypes.c_int()
        _lib.call("mvp_mp4v_decode", ps._h, data.ctypes.data, data.size, out.ctypes.data, None, ctypes.byref(n))
    ps.close()


def test_parse_many_equals_parse_and_stops_before_overflow():
    """mvp_mp4v_parse_many (one native call per GOP) writes what per-sample mvp_mp4v_parse does,
    packed, and stops before a sample that might not fit the coefficient buffer."""
    import ctypes
    cfg, samples, w, h = mixed_stream(4, 3, 3, 21)
    ref = _parse(cfg, samples)
    ps = video.Mp4vParser(cfg)
    n, nmb = len(samples), ps.n_mb
    ptrs = (ctypes.c_char_p * n)(*samples)
    sizes = np.array([len(x) for x in samples], np.uint64)
    rec = np.zeros(n * nmb * 32, np.uint8)
    ncoef = np.zeros(n, np.int64)
    vops = np.zeros((n, 2), np.int32)
    cap = nmb * 384 + 8                  # one worst-case sample: the call stops after the I-VOP
    buf = np.zeros(cap, np.uint32)
    done = ctypes.c_int()
    _lib.call("mvp_mp4v_parse_many", ps._h, n, ptrs, sizes.ctypes.data, rec.ctypes.data, buf.ctypes.data, cap,
              ncoef.ctypes.data, vops.ctypes.data, ctypes.byref(done))
    k = done.value
    assert 1 <= k < n
    off = 0
    for i in range(k):
        r, c, coded, rnd = ref[i]
        assert (vops[i, 0], vops[i, 1]) == (coded, rnd)
        np.testing.assert_array_equal(buf[off:off + ncoef[i]], c)
        if r is not None:
            np.testing.assert_array_equal(rec[i * nmb * 32:(i + 1) * nmb * 32], r)
        off += int(ncoef[i])
    ps.close()
