"""Test infrastructure: an MPEG-4 Part 2 Simple Profile bitstream WRITER and a numpy restatement
of the decoder's reconstruction (inverse quantisation, FFmpeg's simple IDCT, half-pel motion
compensation), for tests/test_mp4v.py.

The writer takes what a decoder must reconstruct — per macroblock the final quantised
coefficients, QP, motion vectors — and emits the VOL / VOP syntax of ISO/IEC 14496-2: intra DC
differentials against the DC prediction, AC prediction residuals, CBP, DQUANT, MV differences
against the median prediction, TCOEF events with their escapes.  Its VLC tables are a separate
transcription of the standard's (the decoder's live in csrc/mp4v_tables.h): a transcription error
on either side fails the round trip.  Prediction rules follow FFmpeg's mpeg4 decoder where the
standard leaves room (slice-edge DC predictors, MV prediction on the first row).
"""
from __future__ import annotations

import numpy as np

# ------------------------------------------------------------------ tables (ISO/IEC 14496-2 annex B)
MCBPC_I = [(1, 1), (1, 3), (2, 3), (3, 3), (1, 4), (1, 6), (2, 6), (3, 6)]          # + 4 for dquant
MCBPC_P = {0: [(1, 1), (3, 4), (2, 4), (5, 6)],        # inter
           4: [(3, 5), (4, 8), (3, 8), (3, 7)],        # intra
           8: [(3, 3), (7, 7), (6, 7), (5, 9)],        # inter + q
           12: [(4, 6), (4, 9), (3, 9), (2, 9)],       # intra + q
           16: [(2, 3), (5, 7), (4, 7), (5, 8)]}       # inter4v
CBPY = [(3, 4), (5, 5), (4, 5), (9, 4), (3, 5), (7, 4), (2, 6), (11, 4),
        (2, 5), (3, 6), (5, 4), (10, 4), (4, 4), (8, 4), (6, 4), (3, 2)]
MVD = [(1, 1), (1, 2), (1, 3), (1, 4), (3, 6), (5, 7), (4, 7), (3, 7), (11, 9), (10, 9), (9, 9), (17, 10),
       (16, 10), (15, 10), (14, 10), (13, 10), (12, 10), (11, 10), (10, 10), (9, 10), (8, 10), (7, 10), (6, 10),
       (5, 10), (4, 10), (7, 11), (6, 11), (5, 11), (4, 11), (3, 11), (2, 11), (3, 12), (2, 12)]
DC_LUM = [(3, 3), (3, 2), (2, 2), (2, 3), (1, 3), (1, 4), (1, 5), (1, 6), (1, 7), (1, 8), (1, 9), (1, 10), (1, 11)]
DC_CHROM = [(3, 2), (2, 2), (1, 2), (1, 3), (1, 4), (1, 5), (1, 6), (1, 7), (1, 8), (1, 9), (1, 10), (1, 11),
            (1, 12)]
ESCAPE = (3, 7)

# TCOEF: {(last, run, level): (code, len)} — Table B-17 (inter) transcribed from the standard's
# (last, run, level) listing; Table B-16 (intra) uses the same codewords for other events.
_INTER_ROWS = [  # (last, run, [codes for level 1..])
    (0, 0, [(0x2, 2), (0xf, 4), (0x15, 6), (0x17, 7), (0x1f, 8), (0x25, 9), (0x24, 9), (0x21, 10), (0x20, 10),
            (0x7, 11), (0x6, 11), (0x20, 11)]),
    (0, 1, [(0x6, 3), (0x14, 6), (0x1e, 8), (0xf, 10), (0x21, 11), (0x50, 12)]),
    (0, 2, [(0xe, 4), (0x1d, 8), (0xe, 10), (0x51, 12)]),
    (0, 3, [(0xd, 5), (0x23, 9), (0xd, 10)]),
    (0, 4, [(0xc, 5), (0x22, 9), (0x52, 12)]),
    (0, 5, [(0xb, 5), (0xc, 10), (0x53, 12)]),
    (0, 6, [(0x13, 6), (0xb, 10), (0x54, 12)]),
    (0, 7, [(0x12, 6), (0xa, 10)]),
    (0, 8, [(0x11, 6), (0x9, 10)]),
    (0, 9, [(0x10, 6), (0x8, 10)]),
    (0, 10, [(0x16, 7), (0x55, 12)]),
] + [(0, r, [c]) for r, c in zip(range(11, 27), [(0x15, 7), (0x14, 7), (0x1c, 8), (0x1b, 8), (0x21, 9), (0x20, 9),
                                                  (0x1f, 9), (0x1e, 9), (0x1d, 9), (0x1c, 9), (0x1b, 9), (0x1a, 9),
                                                  (0x22, 11), (0x23, 11), (0x56, 12), (0x57, 12)])] + [
    (1, 0, [(0x7, 4), (0x19, 9), (0x5, 11)]),
    (1, 1, [(0xf, 6), (0x4, 11)]),
] + [(1, r, [c]) for r, c in zip(range(2, 41), [(0xe, 6), (0xd, 6), (0xc, 6), (0x13, 7), (0x12, 7), (0x11, 7),
                                                 (0x10, 7), (0x1a, 8), (0x19, 8), (0x18, 8), (0x17, 8), (0x16, 8),
                                                 (0x15, 8), (0x14, 8), (0x13, 8), (0x18, 9), (0x17, 9), (0x16, 9),
                                                 (0x15, 9), (0x14, 9), (0x13, 9), (0x12, 9), (0x11, 9), (0x7, 10),
                                                 (0x6, 10), (0x5, 10), (0x4, 10), (0x24, 11), (0x25, 11), (0x26, 11),
                                                 (0x27, 11), (0x58, 12), (0x59, 12), (0x5a, 12), (0x5b, 12),
                                                 (0x5c, 12), (0x5d, 12), (0x5e, 12), (0x5f, 12)])]
_INTRA_ROWS = [
    (0, 0, [(0x2, 2), (0x6, 3), (0xf, 4), (0xd, 5), (0xc, 5), (0x15, 6), (0x13, 6), (0x12, 6), (0x17, 7), (0x1f, 8),
            (0x1e, 8), (0x1d, 8), (0x25, 9), (0x24, 9), (0x23, 9), (0x21, 9), (0x21, 10), (0x20, 10), (0xf, 10),
            (0xe, 10), (0x7, 11), (0x6, 11), (0x20, 11), (0x21, 11), (0x50, 12), (0x51, 12), (0x52, 12)]),
    (0, 1, [(0xe, 4), (0x14, 6), (0x16, 7), (0x1c, 8), (0x20, 9), (0x1f, 9), (0xd, 10), (0x22, 11), (0x53, 12),
            (0x55, 12)]),
    (0, 2, [(0xb, 5), (0x15, 7), (0x1e, 9), (0xc, 10), (0x56, 12)]),
    (0, 3, [(0x11, 6), (0x1b, 8), (0x1d, 9), (0xb, 10)]),
    (0, 4, [(0x10, 6), (0x22, 9), (0xa, 10)]),
    (0, 5, [(0xd, 6), (0x1c, 9), (0x8, 10)]),
    (0, 6, [(0x12, 7), (0x1b, 9), (0x54, 12)]),
    (0, 7, [(0x14, 7), (0x1a, 9), (0x57, 12)]),
    (0, 8, [(0x19, 8), (0x9, 10)]),
    (0, 9, [(0x18, 8), (0x23, 11)]),
    (0, 10, [(0x17, 8)]), (0, 11, [(0x19, 9)]), (0, 12, [(0x18, 9)]), (0, 13, [(0x7, 10)]), (0, 14, [(0x58, 12)]),
    (1, 0, [(0x7, 4), (0xc, 6), (0x16, 8), (0x17, 9), (0x6, 10), (0x5, 11), (0x4, 11), (0x59, 12)]),
    (1, 1, [(0xf, 6), (0x16, 9), (0x5, 10)]),
    (1, 2, [(0xe, 6), (0x4, 10)]), (1, 3, [(0x11, 7), (0x24, 11)]), (1, 4, [(0x10, 7), (0x25, 11)]),
    (1, 5, [(0x13, 7), (0x5a, 12)]), (1, 6, [(0x15, 8), (0x5b, 12)]),
] + [(1, r, [c]) for r, c in zip(range(7, 21), [(0x14, 8), (0x13, 8), (0x1a, 8), (0x15, 9), (0x14, 9), (0x13, 9),
                                                 (0x12, 9), (0x11, 9), (0x26, 11), (0x27, 11), (0x5c, 12),
                                                 (0x5d, 12), (0x5e, 12), (0x5f, 12)])]


def _events(rows):
    return {(last, run, lev + 1): c for last, run, codes in rows for lev, c in enumerate(codes)}


TCOEF = {True: _events(_INTRA_ROWS), False: _events(_INTER_ROWS)}
LMAX = {t: {} for t in (True, False)}
RMAX = {t: {} for t in (True, False)}
for _t, _ev in TCOEF.items():
    for (_last, _run, _lev) in _ev:
        LMAX[_t][(_last, _run)] = max(LMAX[_t].get((_last, _run), 0), _lev)
        RMAX[_t][(_last, _lev)] = max(RMAX[_t].get((_last, _lev), 0), _run)

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                   45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
ALT_H = np.array([0, 1, 2, 3, 8, 9, 16, 17, 10, 11, 4, 5, 6, 7, 15, 14, 13, 12, 19, 18, 24, 25, 32, 33, 26, 27, 20,
                  21, 22, 23, 28, 29, 30, 31, 34, 35, 40, 41, 48, 49, 42, 43, 36, 37, 38, 39, 44, 45, 46, 47, 50,
                  51, 56, 57, 58, 59, 52, 53, 54, 55, 60, 61, 62, 63])
ALT_V = (ALT_H % 8) * 8 + ALT_H // 8


def dc_scale(q, luma):
    if luma:
        return 8 if q < 5 else 2 * q if q < 9 else q + 8 if q < 25 else 2 * q - 16
    return 8 if q < 5 else (q + 13) // 2 if q < 25 else q - 6


# ------------------------------------------------------------------ bits
class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, value, n):
        for i in range(n - 1, -1, -1):
            self.bits.append((value >> i) & 1)

    def code(self, c):
        self.put(*c)

    def stuff(self):
        """MPEG-4 next_start_code stuffing: a 0, then 1s to the byte boundary."""
        self.bits.append(0)
        while len(self.bits) % 8:
            self.bits.append(1)

    def start_code(self, code):
        assert len(self.bits) % 8 == 0
        self.put(0x000001, 24)
        self.put(code, 8)

    def tobytes(self):
        b = self.bits + [0] * (-len(self.bits) % 8)
        return np.packbits(np.array(b, np.uint8)).tobytes()


def vol_header(w, h, quant_type=0, resync_disable=1, time_res=30, intra_matrix=None):
    """VOS + VO + VOL headers as FFmpeg's mpeg4 encoder writes them (object layer id, vol control
    parameters, rectangular, progressive, 8-bit)."""
    bw = BitWriter()
    bw.start_code(0xB0)
    bw.put(1, 8)                  # profile_and_level_indication: simple L1
    bw.start_code(0xB5)
    bw.put(0, 1)                  # is_visual_object_identifier
    bw.put(1, 4)                  # visual_object_type: video
    bw.put(0, 1)                  # video_signal_type
    bw.stuff()
    bw.start_code(0x00)           # video_object_start_code
    bw.start_code(0x20)           # video_object_layer_start_code
    bw.put(0, 1)
    bw.put(1, 8)                  # simple object
    bw.put(1, 1)                  # is_object_layer_identifier
    bw.put(1, 4)                  # verid 1
    bw.put(1, 3)
    bw.put(1, 4)                  # aspect ratio 1:1
    bw.put(1, 1)                  # vol_control_parameters
    bw.put(1, 2)                  # 4:2:0
    bw.put(1, 1)                  # low_delay
    bw.put(0, 1)                  # vbv
    bw.put(0, 2)                  # rectangular
    bw.put(1, 1)
    bw.put(time_res, 16)
    bw.put(1, 1)
    bw.put(0, 1)                  # fixed_vop_rate
    bw.put(1, 1)
    bw.put(w, 13)
    bw.put(1, 1)
    bw.put(h, 13)
    bw.put(1, 1)
    bw.put(0, 1)                  # interlaced
    bw.put(1, 1)                  # obmc_disable
    bw.put(0, 1)                  # sprite
    bw.put(0, 1)                  # not_8_bit
    bw.put(quant_type, 1)
    if quant_type:
        if intra_matrix is None:
            bw.put(0, 1)
        else:
            bw.put(1, 1)
            for v in np.asarray(intra_matrix).reshape(64)[ZIGZAG]:
                bw.put(int(v), 8)
        bw.put(0, 1)              # default inter matrix
    bw.put(1, 1)                  # complexity_estimation_disable
    bw.put(resync_disable, 1)
    bw.put(0, 1)                  # data_partitioned
    bw.put(0, 1)                  # scalability
    bw.stuff()
    return bw.tobytes()


def time_bits(res):
    return max(1, int(res - 1).bit_length())


# ------------------------------------------------------------------ VOP writer
class VopWriter:
    """Writes I / P VOPs of w x h (multiples of 16) and tracks the predictor state a decoder
    builds, so every prediction residual it writes is against the decoder's predictor."""

    def __init__(self, w, h, time_res=30):
        self.w, self.h = w, h
        self.mw, self.mh = w // 16, h // 16
        self.tb = time_bits(time_res)
        self.n = 0

    # --- predictor state, FFmpeg layout semantics
    def _reset(self):
        mw, mh = self.mw, self.mh
        self.dc = [np.full((2 * mh + 1, 2 * mw + 2), 1024, np.int64)] + [np.full((mh + 1, mw + 2), 1024, np.int64)
                                                                       for _ in range(2)]
        self.ac = [np.zeros((2 * mh + 1, 2 * mw + 2, 16), np.int64)] + [np.zeros((mh + 1, mw + 2, 16), np.int64)
                                                                      for _ in range(2)]
        self.mv = np.zeros((2 * mh + 1, 2 * mw + 2, 2), np.int64)
        self.mbq = np.zeros((mh + 1, mw + 2), np.int64)

    def _pos(self, n, x, y):
        if n < 4:
            return 0, 2 * y + (n >> 1) + 1, 2 * x + (n & 1) + 1
        return n - 3, y + 1, x + 1

    def _pred_dc(self, n, x, y, q, first_line):
        p, r, c = self._pos(n, x, y)
        d = self.dc[p]
        a, b, cc = d[r, c - 1], d[r - 1, c - 1], d[r - 1, c]
        if first_line and n != 3:
            if n != 2:
                b = cc = 1024
            if n != 1 and x == 0:
                b = a = 1024
        if x == 0 and y == 1 and n in (0, 4, 5):
            b = 1024
        if abs(a - b) < abs(b - cc):
            pred, direction = cc, 1
        else:
            pred, direction = a, 0
        s = dc_scale(q, n < 4)
        return (int(pred) + (s >> 1)) // s, direction

    def _ac_pred_values(self, n, x, y, q, direction):
        """The predicted first column (direction 0) or first row (1), quantised domain."""
        p, r, c = self._pos(n, x, y)
        out = np.zeros(8, np.int64)
        if direction == 0:
            src = self.ac[p][r, c - 1]
            ql = self.mbq[y + 1, x]
            same = x == 0 or q == ql or n in (1, 3)
            for i in range(1, 8):
                out[i] = src[i] if same else _rdiv(src[i] * ql, q)
        else:
            src = self.ac[p][r - 1, c]
            qt = self.mbq[y, x + 1]
            same = y == 0 or q == qt or n in (2, 3)
            for i in range(1, 8):
                out[i] = src[8 + i] if same else _rdiv(src[8 + i] * qt, q)
        return out

    def _store_intra(self, n, x, y, q, blk):
        p, r, c = self._pos(n, x, y)
        level = int(blk[0]) * dc_scale(q, n < 4)
        if level & ~2047:
            level = 0 if level < 0 else 2047
        self.dc[p][r, c] = level
        a = self.ac[p][r, c]
        a[:] = 0
        for i in range(1, 8):
            a[i] = blk[i * 8]
            a[8 + i] = blk[i]

    def _clear_intra(self, x, y):
        for n in range(6):
            p, r, c = self._pos(n, x, y)
            self.dc[p][r, c] = 1024
            self.ac[p][r, c] = 0

    # --- syntax
    def _header(self, bw, vtype, q, rounding=0, fcode=1):
        bw.start_code(0xB6)
        bw.put(vtype, 2)
        bw.put(0, 1)               # modulo_time_base
        bw.put(1, 1)
        bw.put(self.n % (1 << self.tb), self.tb)
        bw.put(1, 1)
        bw.put(1, 1)               # vop_coded
        if vtype == 1:
            bw.put(rounding, 1)
        bw.put(0, 3)               # intra_dc_vlc_thr: always the DC VLC
        bw.put(q, 5)
        if vtype == 1:
            bw.put(fcode, 3)
        self.n += 1

    def _tcoef(self, bw, coefs, intra):
        """coefs: (run, level) pairs in scan order, the last flagged implicitly."""
        ev = TCOEF[intra]
        for k, (run, level) in enumerate(coefs):
            last = int(k == len(coefs) - 1)
            a, s = abs(level), int(level < 0)
            if (last, run, a) in ev:
                bw.code(ev[(last, run, a)])
                bw.put(s, 1)
                continue
            lm = LMAX[intra].get((last, run), 0)
            if lm and (last, run, a - lm) in ev:              # escape type 1
                bw.code(ESCAPE)
                bw.put(0, 1)
                bw.code(ev[(last, run, a - lm)])
                bw.put(s, 1)
                continue
            rm = RMAX[intra].get((last, a), None)
            if rm is not None and (last, run - rm - 1, a) in ev:  # escape type 2
                bw.code(ESCAPE)
                bw.put(2, 2)
                bw.code(ev[(last, run - rm - 1, a)])
                bw.put(s, 1)
                continue
            bw.code(ESCAPE)                                   # type 3
            bw.put(3, 2)
            bw.put(last, 1)
            bw.put(run, 6)
            bw.put(1, 1)
            bw.put(level & 0xFFF, 12)
            bw.put(1, 1)

    @staticmethod
    def _runs(blk, scan, start):
        out, run = [], 0
        for i in range(start, 64):
            v = int(blk[scan[i]])
            if v == 0:
                run += 1
            else:
                out.append((run, v))
                run = 0
        return out

    def _intra_mb(self, bw, x, y, mb, q, first_line, p_vop):
        """mb: {"blocks": (6, 64) final quantised coefficients (raster), "ac_pred": bool}"""
        blocks = np.asarray(mb["blocks"], np.int64).reshape(6, 64)
        ac_pred = bool(mb.get("ac_pred", False))
        trans, dcs = [], []
        for n in range(6):
            pred, direction = self._pred_dc(n, x, y, q, first_line)
            blk = blocks[n].copy()
            t = blk.copy()
            if ac_pred:
                pv = self._ac_pred_values(n, x, y, q, direction)
                if direction == 0:
                    for i in range(1, 8):
                        t[i * 8] -= pv[i]
                else:
                    for i in range(1, 8):
                        t[i] -= pv[i]
            scan = (ALT_V if direction == 0 else ALT_H) if ac_pred else ZIGZAG
            dcs.append(int(blk[0]) - pred)
            trans.append(self._runs(t, scan, 1))
            self._store_intra(n, x, y, q, blk)
        cbp = sum(1 << (5 - n) for n in range(6) if trans[n])
        return ac_pred, cbp, dcs, trans

    def _write_intra_blocks(self, bw, dcs, trans):
        for n in range(6):
            d = dcs[n]
            size = abs(d).bit_length()
            assert size <= 12, d
            bw.code((DC_LUM if n < 4 else DC_CHROM)[size])
            if size:
                bw.put(d if d > 0 else d + (1 << size) - 1, size)
                if size > 8:
                    bw.put(1, 1)
            if trans[n]:
                self._tcoef(bw, trans[n], True)

    def i_vop(self, mbs, q0):
        """mbs[y][x] = {"q": QP (within 2 of the previous MB's), "blocks": (6, 64), "ac_pred": bool}"""
        self._reset()
        bw = BitWriter()
        self._header(bw, 0, q0)
        q = q0
        for y in range(self.mh):
            for x in range(self.mw):
                mb = mbs[y][x]
                qn = mb.get("q", q)
                dq = qn - q
                assert dq in (0, -1, -2, 1, 2)
                ac_pred, cbp, dcs, trans = self._intra_mb(bw, x, y, mb, qn, y == 0, False)
                bw.code(MCBPC_I[(cbp & 3) + (4 if dq else 0)])
                bw.put(int(ac_pred), 1)
                bw.code(CBPY[cbp >> 2])
                if dq:
                    bw.put({-1: 0, -2: 1, 1: 2, 2: 3}[dq], 2)
                q = qn
                self.mbq[y + 1, x + 1] = q
                self._write_intra_blocks(bw, dcs, trans)
        bw.stuff()
        return bw.tobytes()

    # --- motion vectors
    def _mvslot(self, x, y, k):
        return 2 * y + (k >> 1) + 1, 2 * x + (k & 1) + 1

    def _pred_mv(self, x, y, k, first_line):
        off = {0: 2, 1: 1, 2: 1, 3: -1}[k]
        r, c = self._mvslot(x, y, k)
        A = self.mv[r, c - 1]
        if first_line and k < 3:
            if k == 0:
                return (0, 0) if x == 0 else tuple(A)
            if k == 1:
                return tuple(A)
            B, C = self.mv[r - 1, c], self.mv[r - 1, c + off]
            if x == 0:
                self.mv[r, c - 1] = 0
                A = self.mv[r, c - 1]
            return tuple(int(np.median([A[i], B[i], C[i]])) for i in range(2))
        B, C = self.mv[r - 1, c], self.mv[r - 1, c + off]
        return tuple(int(np.median([A[i], B[i], C[i]])) for i in range(2))

    @staticmethod
    def _mvd(bw, diff, fcode):
        shift = fcode - 1
        rng = 32 << shift
        diff = ((diff + rng) % (2 * rng)) - rng    # wrap into the representable range
        if diff == 0:
            bw.code(MVD[0])
            return
        a = abs(diff) - 1
        code = (a >> shift) + 1
        bw.code(MVD[code])
        bw.put(int(diff < 0), 1)
        if shift:
            bw.put(a & ((1 << shift) - 1), shift)

    def p_vop(self, mbs, q0, rounding=0, fcode=1):
        """mbs[y][x] = {"type": "skip"} | {"type": "inter", "mv": (x, y)} |
        {"type": "inter4v", "mvs": [(x, y)] * 4} | {"type": "intra", ...i_vop fields}; inter types
        take "q" and "blocks" (6, 64) quantised residual coefficients (raster)."""
        self.mv[:] = 0
        bw = BitWriter()
        self._header(bw, 1, q0, rounding, fcode)
        q = q0
        for y in range(self.mh):
            for x in range(self.mw):
                mb = mbs[y][x]
                first = y == 0
                t = mb["type"]
                if t == "skip":
                    bw.put(1, 1)
                    self._clear_intra(x, y)
                    for k in range(4):
                        self.mv[self._mvslot(x, y, k)] = 0
                    self.mbq[y + 1, x + 1] = q
                    continue
                bw.put(0, 1)
                qn = mb.get("q", q)
                dq = qn - q
                assert dq in (0, -1, -2, 1, 2)
                if t == "intra":
                    for k in range(4):
                        self.mv[self._mvslot(x, y, k)] = 0
                    ac_pred, cbp, dcs, trans = self._intra_mb(bw, x, y, mb, qn, first, True)
                    bw.code(MCBPC_P[12 if dq else 4][cbp & 3])
                    bw.put(int(ac_pred), 1)
                    bw.code(CBPY[cbp >> 2])
                    if dq:
                        bw.put({-1: 0, -2: 1, 1: 2, 2: 3}[dq], 2)
                    q = qn
                    self.mbq[y + 1, x + 1] = q
                    self._write_intra_blocks(bw, dcs, trans)
                    continue
                self._clear_intra(x, y)
                blocks = np.asarray(mb.get("blocks", np.zeros((6, 64))), np.int64).reshape(6, 64)
                trans = [self._runs(blocks[n], ZIGZAG, 0) for n in range(6)]
                cbp = sum(1 << (5 - n) for n in range(6) if trans[n])
                four = t == "inter4v"
                assert not (four and dq), "inter4v + q is not Simple Profile"
                bw.code(MCBPC_P[(16 if four else 8 if dq else 0)][cbp & 3])
                bw.code(CBPY[15 - (cbp >> 2)])
                if dq:
                    bw.put({-1: 0, -2: 1, 1: 2, 2: 3}[dq], 2)
                q = qn
                self.mbq[y + 1, x + 1] = q
                mvs = mb["mvs"] if four else [mb["mv"]] * 4
                for k in range(4 if four else 1):
                    px, py = self._pred_mv(x, y, k, first)
                    self._mvd(bw, mvs[k][0] - px, fcode)
                    self._mvd(bw, mvs[k][1] - py, fcode)
                    if four:
                        self.mv[self._mvslot(x, y, k)] = mvs[k]
                if not four:
                    for k in range(4):
                        self.mv[self._mvslot(x, y, k)] = mvs[0]
                for n in range(6):
                    if trans[n]:
                        self._tcoef(bw, trans[n], False)
        bw.stuff()
        return bw.tobytes()


def _rdiv(a, b):
    a, b = int(a), int(b)
    return int((a + (b >> 1)) // b) if a >= 0 else -int((-a + (b >> 1)) // b)


# ------------------------------------------------------------------ reconstruction restated
W1, W2, W3, W4, W5, W6, W7 = 22725, 21407, 19266, 16383, 12873, 8867, 4520


def simple_idct(blk):
    """FFmpeg's simple IDCT (8-bit), restated in numpy int64: rows (DC-only shortcut x 8, else
    shift 11 with rounding), then columns (shift 20, W4 x (c0 + 32) rounding)."""
    b = np.asarray(blk, np.int64).reshape(8, 8).copy()
    for r in range(8):
        x = b[r]
        if not x[1:].any():
            v = (int(x[0]) * 8) & 0xFFFF          # the DC-only shortcut, stored as int16
            b[r] = v - 65536 if v >= 32768 else v
            continue
        a0 = W4 * x[0] + (1 << 10)
        a1, a2, a3 = a0, a0, a0
        a0, a1, a2, a3 = a0 + W2 * x[2], a1 + W6 * x[2], a2 - W6 * x[2], a3 - W2 * x[2]
        b0 = W1 * x[1] + W3 * x[3]
        b1 = W3 * x[1] - W7 * x[3]
        b2 = W5 * x[1] - W1 * x[3]
        b3 = W7 * x[1] - W5 * x[3]
        a0 += W4 * x[4] + W6 * x[6]
        a1 += -W4 * x[4] - W2 * x[6]
        a2 += -W4 * x[4] + W2 * x[6]
        a3 += W4 * x[4] - W6 * x[6]
        b0 += W5 * x[5] + W7 * x[7]
        b1 += -W1 * x[5] - W5 * x[7]
        b2 += W7 * x[5] + W3 * x[7]
        b3 += W3 * x[5] - W1 * x[7]
        row = np.array([a0 + b0, a1 + b1, a2 + b2, a3 + b3, a3 - b3, a2 - b2, a1 - b1, a0 - b0], np.int64) >> 11
        b[r] = ((row + 32768) & 0xFFFF) - 32768   # int16 storage
    out = np.empty((8, 8), np.int64)
    for c in range(8):
        x = b[:, c]
        a0 = W4 * (x[0] + ((1 << 19) // W4))
        a1, a2, a3 = a0, a0, a0
        a0, a1, a2, a3 = a0 + W2 * x[2], a1 + W6 * x[2], a2 - W6 * x[2], a3 - W2 * x[2]
        b0 = W1 * x[1] + W3 * x[3]
        b1 = W3 * x[1] - W7 * x[3]
        b2 = W5 * x[1] - W1 * x[3]
        b3 = W7 * x[1] - W5 * x[3]
        a0, a1, a2, a3 = a0 + W4 * x[4], a1 - W4 * x[4], a2 - W4 * x[4], a3 + W4 * x[4]
        b0, b1, b2, b3 = b0 + W5 * x[5], b1 - W1 * x[5], b2 + W7 * x[5], b3 + W3 * x[5]
        a0, a1, a2, a3 = a0 + W6 * x[6], a1 - W2 * x[6], a2 + W2 * x[6], a3 - W6 * x[6]
        b0, b1, b2, b3 = b0 + W7 * x[7], b1 - W5 * x[7], b2 + W3 * x[7], b3 - W1 * x[7]
        out[:, c] = np.array([a0 + b0, a1 + b1, a2 + b2, a3 + b3, a3 - b3, a2 - b2, a1 - b1, a0 - b0]) >> 20
    return out


def float_idct(blk):
    """The separable 8x8 inverse DCT in float64 (IEEE 1180 reference)."""
    k = np.arange(8)
    cu = np.where(k == 0, np.sqrt(0.125), 0.5)
    basis = cu[:, None] * np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16)   # [u, x]
    return basis.T @ np.asarray(blk, np.float64).reshape(8, 8) @ basis


def dequant_h263(blk, q, intra, luma=True):
    b = np.asarray(blk, np.int64).reshape(64).copy()
    qmul, qadd = 2 * q, (q - 1) | 1
    start = 1 if intra else 0
    for i in range(start, 64):
        v = b[i]
        if v:
            b[i] = max(-2048, min(2047, v * qmul - qadd if v < 0 else v * qmul + qadd))
    if intra:
        b[0] = b[0] * dc_scale(q, luma)
    return b


def mc_plane(ref, x0, y0, w, h, mvx, mvy, rnd):
    """Half-pel prediction of a w x h block at (x0, y0) with edge clamping (unrestricted MVs)."""
    H, W = ref.shape
    sx, sy = x0 + (mvx >> 1), y0 + (mvy >> 1)
    ys = np.clip(np.arange(sy, sy + h + 1), 0, H - 1)
    xs = np.clip(np.arange(sx, sx + w + 1), 0, W - 1)
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


def chroma_mv(v):
    return (v >> 1) | (v & 1)


def chroma_mv4(s):
    tab = [0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2]
    return tab[s & 15] + ((s >> 3) & ~1)


def reconstruct(w, h, vops, fcode=1):
    """The expected I420 planes of each VOP spec [(kind, mbs, q0, rounding)] (numpy)."""
    frames, ref = [], None
    for kind, mbs, q0, rnd in vops:
        planes = [np.zeros((h, w), np.int64), np.zeros((h // 2, w // 2), np.int64), np.zeros((h // 2, w // 2), np.int64)]
        q = q0
        for y in range(h // 16):
            for x in range(w // 16):
                mb = mbs[y][x]
                t = mb.get("type", "intra")
                q = mb.get("q", q)
                if t == "skip":
                    for pl, sz in ((0, 16), (1, 8), (2, 8)):
                        planes[pl][sz * y:sz * y + sz, sz * x:sz * x + sz] = ref[pl][sz * y:sz * y + sz, sz * x:sz * x + sz]
                    continue
                blocks = np.asarray(mb.get("blocks", np.zeros((6, 64))), np.int64).reshape(6, 64)
                pred = None
                if t in ("inter", "inter4v"):
                    mvs = mb["mvs"] if t == "inter4v" else [mb["mv"]] * 4
                    lp = np.zeros((16, 16), np.int64)
                    if t == "inter4v":
                        for k in range(4):
                            lp[8 * (k >> 1):8 * (k >> 1) + 8, 8 * (k & 1):8 * (k & 1) + 8] = mc_plane(
                                ref[0], 16 * x + 8 * (k & 1), 16 * y + 8 * (k >> 1), 8, 8, mvs[k][0], mvs[k][1], rnd)
                        cx = chroma_mv4(sum(m[0] for m in mvs))
                        cy = chroma_mv4(sum(m[1] for m in mvs))
                    else:
                        lp = mc_plane(ref[0], 16 * x, 16 * y, 16, 16, mvs[0][0], mvs[0][1], rnd)
                        cx, cy = chroma_mv(mvs[0][0]), chroma_mv(mvs[0][1])
                    pred = [lp] + [mc_plane(ref[c], 8 * x, 8 * y, 8, 8, cx, cy, rnd) for c in (1, 2)]
                for n in range(6):
                    intra = pred is None
                    deq = dequant_h263(blocks[n], q, intra, n < 4)
                    res = simple_idct(deq) if (intra or blocks[n].any()) else np.zeros((8, 8), np.int64)
                    if n < 4:
                        pl, oy, ox = 0, 16 * y + 8 * (n >> 1), 16 * x + 8 * (n & 1)
                        base = None if intra else pred[0][8 * (n >> 1):8 * (n >> 1) + 8, 8 * (n & 1):8 * (n & 1) + 8]
                    else:
                        pl, oy, ox = n - 3, 8 * y, 8 * x
                        base = None if intra else pred[n - 3]
                    val = res if intra else base + res
                    planes[pl][oy:oy + 8, ox:ox + 8] = np.clip(val, 0, 255)
        ref = planes
        frames.append([p.astype(np.uint8) for p in planes])
    return frames


# ------------------------------------------------------------------ containers
def _box(kind, body):
    import struct
    return struct.pack(">I4s", 8 + len(body), kind) + body


def _desc(tag, body):
    n = len(body)
    return bytes([tag, 0x80 | (n >> 21) & 0x7F, 0x80 | (n >> 14) & 0x7F, 0x80 | (n >> 7) & 0x7F, n & 0x7F]) + body


def mp4_file(config, samples, w, h, fps=30, chunk=3):
    """A minimal ISO BMFF file: ftyp, moov (one 'vide' track with an 'mp4v' sample entry whose
    esds carries `config`; samples grouped `chunk` per chunk through stsc / stco / stsz), mdat."""
    import struct
    esds = _box(b"esds", b"\0\0\0\0" + _desc(0x03, struct.pack(">HB", 1, 0) + _desc(
        0x04, bytes([0x20, 0x11]) + b"\0\0\0" + struct.pack(">II", 0, 0) + _desc(0x05, config)) + _desc(0x06, b"\x02")))
    entry = (b"\0" * 6 + struct.pack(">H", 1) + b"\0" * 16 + struct.pack(">HH", w, h) +
             struct.pack(">IIIH", 0x480000, 0x480000, 0, 1) + b"\0" * 32 + struct.pack(">Hh", 24, -1) + esds)
    stsd = _box(b"stsd", struct.pack(">II", 0, 1) + _box(b"mp4v", entry))
    stts = _box(b"stts", struct.pack(">III", 0, 1, len(samples)) + struct.pack(">I", 1000))
    n_chunks = (len(samples) + chunk - 1) // chunk
    stsc_rows = [(1, chunk, 1)]
    if len(samples) % chunk:
        stsc_rows.append((n_chunks, len(samples) % chunk, 1))
    stsc = _box(b"stsc", struct.pack(">II", 0, len(stsc_rows)) + b"".join(struct.pack(">III", *r) for r in stsc_rows))
    stsz = _box(b"stsz", struct.pack(">III", 0, 0, len(samples)) + b"".join(struct.pack(">I", len(s)) for s in samples))
    mdhd = _box(b"mdhd", struct.pack(">IIIIIHH", 0, 0, 0, int(fps * 1000), len(samples) * 1000, 0, 0))
    hdlr = _box(b"hdlr", struct.pack(">II4s", 0, 0, b"vide") + b"\0" * 12 + b"VideoHandler\0")

    def build(chunk_offsets):
        stco = _box(b"stco", struct.pack(">II", 0, len(chunk_offsets)) + b"".join(struct.pack(">I", o)
                                                                                  for o in chunk_offsets))
        stbl = _box(b"stbl", stsd + stts + stsc + stsz + stco)
        minf = _box(b"minf", _box(b"vmhd", struct.pack(">IHHHH", 1, 0, 0, 0, 0)) + stbl)
        mdia = _box(b"mdia", mdhd + hdlr + minf)
        trak = _box(b"trak", _box(b"tkhd", struct.pack(">II", 3, 0) + b"\0" * 76 + struct.pack(">II", w << 16, h << 16))
                    + mdia)
        return _box(b"moov", _box(b"mvhd", b"\0" * 100) + trak)

    ftyp = _box(b"ftyp", b"isom\0\0\x02\0isomiso2mp41")
    moov = build([0] * n_chunks)
    base = len(ftyp) + len(moov) + 8
    offs, o = [], base
    for i, s in enumerate(samples):
        if i % chunk == 0:
            offs.append(o)
        o += len(s)
    moov = build(offs)
    return ftyp + moov + _box(b"mdat", b"".join(samples))
