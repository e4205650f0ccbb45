"""Recording ingest: the reference's frame_generator / read_video_as_frames
(utils.py:849-909) decode a whole recording with cv2.VideoCapture into a list of BGR frames
before slicing [start:end].  This image has no video codec library (no cv2, ffmpeg, PyAV,
rocDecode), so the containers whose codecs ARE available are read here:

* AVI (RIFF, including OpenDML 'AVIX' extensions) with Motion-JPEG video: the frames'
  JPEG bitstreams are located by walking the 'movi' lists and decoded by libjpeg (through
  PIL) on a thread pool; uncompressed 24-bit DIB frames ('BI_RGB', bottom-up rows) are
  copied out exactly.
* Directories of "frame<N>.jpg" files, ordered by N (the reference's
  process_image_files, utils.py:851-860).
* .npy (T, H, W, 3) uint8 stacks, memory-mapped (the build's own recording format).
* MPEG-4 Part 2 ('mp4v') video — what the reference's synchronize_videos.py:64,240 writes
  with cv2.VideoWriter_fourcc(*'mp4v') — in MP4 / QuickTime containers (ISO BMFF: the
  'mp4v' sample entry's esds decoder config, stsc / stco / stsz sample tables), in AVI
  (XVID / DIVX / DX50 / FMP4 / MP4V FourCCs) and as raw elementary streams (.m4v / .cmp),
  decoded by the native Simple Profile decoder in libmvpose.so (csrc/mp4v.cpp; host code).

Every reader returns (T, H, W, 3) uint8 frames in the channel order cv2 returns them
(BGR), so the rest of the pipeline applies the reference's cvtColor(RGB2BGR) swap exactly
as for decoded video.  H.264 / HEVC (QuickTime's usual .mov codecs, record_from_webcams_
with_quicktime.py:39) raise NotImplementedError: this image has no decoder for them.  Decoded
pixels are libjpeg's for MJPEG (islow IDCT, fancy upsampling), which is what cv2.imread uses;
cv2's VideoCapture decodes MJPEG and MPEG-4 with FFmpeg, which is absent here, so parity of
both with the reference is unpinned.
"""
from __future__ import annotations

import io
import mmap
import os
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_BI_RGB = 0
_MJPG = (b"MJPG", b"mjpg", b"AVRn", b"LJPG", b"JPGL", b"dmb1")
_MP4V = (b"XVID", b"xvid", b"DIVX", b"divx", b"DX50", b"dx50", b"FMP4", b"fmp4", b"MP4V", b"mp4v", b"M4S2", b"m4s2")


class AviInfo:
    """Stream 0 of an AVI: frame size, codec, and the (offset, size) of every frame chunk."""

    def __init__(self, width, height, codec, bit_count, fps, chunks):
        self.width, self.height, self.codec, self.bit_count = width, height, codec, bit_count
        self.fps = fps
        self.chunks = chunks

    def __len__(self):
        return len(self.chunks)


def _walk(buf, start, end, visit):
    """Visit every chunk of [start, end): visit(fourcc, list_type or None, data_start, size)
    descends into LISTs / RIFFs whose visit() returns True."""
    p = start
    while p + 8 <= end:
        fourcc = bytes(buf[p:p + 4])
        size = struct.unpack_from("<I", buf, p + 4)[0]
        data = p + 8
        is_list = fourcc in (b"RIFF", b"LIST")
        if data + size > end:          # truncated recording: keep the complete chunks
            if not is_list:
                break
            size = max(0, end - data)
        if is_list and size >= 4:
            kind = bytes(buf[data:data + 4])
            if visit(fourcc, kind, data + 4, size - 4):
                _walk(buf, data + 4, data + size, visit)
        else:
            visit(fourcc, None, data, size)
        p = data + size + (size & 1)   # chunks are word aligned


def parse_avi(buf) -> AviInfo:
    """Parse an AVI held in `buf` (bytes / mmap) -> AviInfo of its first video stream."""
    if len(buf) < 12 or bytes(buf[0:4]) != b"RIFF" or bytes(buf[8:12]) != b"AVI ":
        raise ValueError("not an AVI (RIFF 'AVI ') file")
    st = {"strh": [], "strf": [], "chunks": [], "stream": -1, "fps": 0.0}

    def visit(fourcc, kind, data, size):
        if kind is not None:
            return kind in (b"AVI ", b"AVIX", b"hdrl", b"strl", b"movi", b"rec ")
        if fourcc == b"strh":
            st["strh"].append((data, size))
        elif fourcc == b"strf":
            st["strf"].append((data, size))
        elif len(fourcc) == 4 and fourcc[2:4] in (b"dc", b"db") and fourcc[0:2].isdigit():
            sid = int(fourcc[0:2])
            if st["stream"] < 0:
                st["stream"] = sid
            if sid == st["stream"] and size > 0:
                st["chunks"].append((data, size))
        return False

    _walk(buf, 0, len(buf), visit)
    vid = None
    for i, (d, n) in enumerate(st["strh"]):
        if bytes(buf[d:d + 4]) == b"vids":
            vid = i
            break
    if vid is None or vid >= len(st["strf"]):
        raise ValueError("AVI has no video stream header")
    d, _ = st["strh"][vid]
    handler = bytes(buf[d + 4:d + 8])
    scale, rate = struct.unpack_from("<II", buf, d + 20)
    fd, _ = st["strf"][vid]
    _, width, height, _, bit_count, comp = struct.unpack_from("<IiiHHI", buf, fd)
    comp_cc = struct.pack("<I", comp)
    codec = "rgb" if comp == _BI_RGB else ("mjpeg" if comp_cc in _MJPG or handler in _MJPG else
                                          "mp4v" if comp_cc in _MP4V or handler in _MP4V else
                                          comp_cc.decode("latin-1"))
    info = AviInfo(width, height, codec, bit_count, rate / scale if scale else 0.0, st["chunks"])
    info.strf_extra = bytes(buf[fd + 40:fd + n_strf]) if (n_strf := st["strf"][vid][1]) > 40 else b""
    return info


def _decode_jpeg(data: bytes) -> np.ndarray:
    from PIL import Image
    im = Image.open(io.BytesIO(data))
    rgb = np.asarray(im.convert("RGB"))
    return rgb[:, :, ::-1]             # BGR, as cv2 returns frames


def _mp4v(config, samples, start, end, device):
    """decode_mp4v on the host, or with device set the split decode (decode_mp4v_device)."""
    if device is None:
        return decode_mp4v(config, samples, start, end)
    return decode_mp4v_device(config, samples, start, end, device=device)


def read_avi(path, start=0, end=None, threads=None, device=None):
    """Frames [start:end) of an MJPEG / uncompressed AVI -> (T, H, W, 3) uint8 BGR (mp4v streams
    with device set: a tensor on that device, reconstructed there)."""
    with open(path, "rb") as f:
        buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            info = parse_avi(buf)
            chunks = info.chunks[slice(start, end)]
            H, W = abs(info.height), info.width
            out = np.empty((len(chunks), H, W, 3), np.uint8)
            if info.codec == "rgb":
                if info.bit_count != 24:
                    raise NotImplementedError(f"{path}: {info.bit_count}-bit uncompressed AVI")
                stride = (W * 3 + 3) & ~3
                for i, (d, n) in enumerate(chunks):
                    if n < stride * H:
                        raise ValueError(f"{path}: frame {i} truncated")
                    rows = np.frombuffer(buf[d:d + stride * H], np.uint8).reshape(H, stride)[:, :W * 3]
                    out[i] = (rows[::-1] if info.height > 0 else rows).reshape(H, W, 3)   # DIB rows are BGR
            elif info.codec == "mp4v":
                return _mp4v(info.strf_extra, (bytes(buf[d:d + n]) for d, n in info.chunks), start, end, device)
            elif info.codec == "mjpeg":
                datas = [bytes(buf[d:d + n]) for d, n in chunks]
                workers = max(1, min(int(threads or os.cpu_count() or 1), 16))

                def dec(i):
                    fr = _decode_jpeg(datas[i])
                    if fr.shape != (H, W, 3):
                        raise ValueError(f"{path}: frame {i} is {fr.shape}, stream header says {(H, W, 3)}")
                    out[i] = fr

                with ThreadPoolExecutor(workers) as pool:   # libjpeg releases the GIL
                    list(pool.map(dec, range(len(datas))))
            else:
                raise NotImplementedError(f"{path}: AVI codec {info.codec!r} (only MJPEG and uncompressed "
                                          "24-bit frames can be decoded in this image)")
            return out
        finally:
            buf.close()


def read_image_dir(path, start=0, end=None, threads=None) -> np.ndarray:
    """The reference's process_image_files (utils.py:851-860): *.jpg files of `path`
    ordered by the integer after "frame", sliced [start:end) -> (T, H, W, 3) uint8 BGR."""
    names = [f for f in os.listdir(path) if f.endswith("jpg")]
    names.sort(key=lambda x: int(x.split("frame")[1].split(".")[0]))
    names = names[slice(start, end)]
    if not names:
        return np.empty((0, 0, 0, 3), np.uint8)
    workers = max(1, min(int(threads or os.cpu_count() or 1), 16))

    def load(n):
        with open(os.path.join(path, n), "rb") as f:
            return _decode_jpeg(f.read())

    with ThreadPoolExecutor(workers) as pool:
        frames = list(pool.map(load, names))
    if len({fr.shape for fr in frames}) != 1:
        raise ValueError(f"{path}: frames of different sizes")
    return np.stack(frames)


def read_recording(path, start=0, end=-1, device=None):
    """One camera's recording, sliced [start:end] with Python semantics (the reference's
    default [0, -1] drops the last frame) -> (T, H, W, 3) uint8 BGR (memory-mapped for .npy).
    device: MPEG-4 Part 2 recordings are then split-decoded — entropy decoding on the host,
    reconstruction on the GPU (decode_mp4v_device) — and come back as a tensor on that device
    (bit-identical frames); other formats still return host arrays."""
    p = str(path)
    if os.path.isdir(p):
        return read_image_dir(p, start, end)
    low = p.lower()
    if low.endswith(".npy"):
        arr = np.load(p, mmap_mode="r")
        if arr.dtype != np.uint8 or arr.ndim != 4 or arr.shape[-1] != 3:
            raise ValueError(f"{p}: expected (T, H, W, 3) uint8 frames, got {arr.shape} {arr.dtype}")
        return arr[start:end]
    if not os.path.exists(p):
        raise FileNotFoundError(f"Error loading video: {p}")
    with open(p, "rb") as f:
        head = f.read(12)
    if head[0:4] == b"RIFF" and head[8:12] == b"AVI ":
        return read_avi(p, start, end, device=device)
    if head[4:8] in (b"ftyp", b"moov", b"mdat", b"free", b"wide", b"skip"):
        return read_mp4(p, start, end, device=device)
    if head[0:3] == b"\0\0\1" and (head[3] in (0xB0, 0xB3, 0xB5, 0xB6) or head[3] <= 0x2F):
        return read_m4v(p, start, end, device=device)
    raise NotImplementedError(
        f"{p}: no decoder for this container/codec in this image (MPEG-4 Part 2 in MP4/MOV/AVI/raw, MJPEG and "
        "uncompressed AVI, frame*.jpg directories and .npy stacks are supported)")


# ------------------------------------------------------------------ MPEG-4 Part 2 ('mp4v')
class Mp4vDecoder:
    """The native Simple Profile decoder (mvp_mp4v_*, csrc/mp4v.cpp): feed the decoder config (VOL
    headers), then one sample at a time; each call returns the frame after the sample's last VOP."""

    def __init__(self, config: bytes):
        import ctypes
        from . import _lib
        self._lib = _lib
        self._h = ctypes.c_void_p()
        w, h = ctypes.c_int(), ctypes.c_int()
        cfg = (ctypes.c_uint8 * max(1, len(config))).from_buffer_copy(config or b"\0")
        _lib.call("mvp_mp4v_create", cfg, len(config), ctypes.byref(self._h), ctypes.byref(w), ctypes.byref(h))
        self.width, self.height = w.value, h.value

    def decode(self, sample: bytes, yuv: bool = False, out: np.ndarray | None = None) -> np.ndarray:
        """One sample -> the frame after its last VOP: (H, W, 3) BGR, or the I420 planes with
        yuv=True; out: a C-contiguous uint8 array of that shape to decode into."""
        import ctypes
        data = np.frombuffer(sample, np.uint8)
        n = ctypes.c_int()
        if yuv:
            cw, ch = (self.width + 1) // 2, (self.height + 1) // 2
            size = self.width * self.height + 2 * cw * ch
            if out is None:
                out = np.empty(size, np.uint8)
            if out.dtype != np.uint8 or out.size != size or not out.flags.c_contiguous:
                raise ValueError(f"out must be a C-contiguous uint8 array of {size} bytes (I420 planes)")
            self._lib.call("mvp_mp4v_decode", self._h, data.ctypes.data, data.size, None, out.ctypes.data,
                           ctypes.byref(n))
            return out
        if out is None:
            out = np.empty((self.height, self.width, 3), np.uint8)
        if out.shape != (self.height, self.width, 3) or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous ({self.height}, {self.width}, 3) uint8 array")
        self._lib.call("mvp_mp4v_decode", self._h, data.ctypes.data, data.size, out.ctypes.data, None,
                       ctypes.byref(n))
        return out

    def close(self):
        if self._h:
            self._lib.call("mvp_mp4v_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def split_vops(stream: bytes):
    """An elementary stream -> (config = everything before the first VOP, [samples]).  A sample
    runs from the end of the previous VOP's payload (its next start code) to the end of its own
    VOP's payload, so GOV headers or a repeated VOL travel with the VOP that follows them."""
    idx = []
    i = stream.find(b"\0\0\1")
    while i >= 0:
        idx.append(i)
        i = stream.find(b"\0\0\1", i + 3)
    vops = [i for i in idx if i + 3 < len(stream) and stream[i + 3] == 0xB6]
    if not vops:
        return stream, []
    ends = []
    for v in vops:
        nxt = next((j for j in idx if j > v), len(stream))
        ends.append(nxt)
    samples = [stream[vops[0]:ends[0]]] + [stream[ends[k - 1]:ends[k]] for k in range(1, len(vops))]
    return stream[:vops[0]], samples


def vop_coding_type(sample) -> int:
    """vop_coding_type of the sample's first VOP (0 I, 1 P, 2 B, 3 S), -1 if it holds none."""
    data = bytes(sample)
    i = data.find(b"\0\0\1\xb6")
    return data[i + 4] >> 6 if 0 <= i and i + 4 < len(data) else -1


def decode_mp4v(config: bytes, samples, start=0, end=None, threads=None) -> np.ndarray:
    """Decode frames [start:end) of a sample sequence.  P-VOPs need their predecessors back to
    the last I-VOP, so the sequence splits into independent GOPs (each starting at an I-VOP);
    the GOPs that hold wanted frames decode on a thread pool, one decoder each (the native
    decoder releases the GIL), straight into the output array."""
    samples = list(samples)
    if not config and samples:
        config = samples[0]       # VOL headers in the first sample (AVI without strf extra data)
    keep = range(len(samples))[slice(start, end)]
    lo, hi = (keep.start, keep.stop) if len(keep) and keep.step == 1 else (0, 0)
    probe = Mp4vDecoder(config)
    H, W = probe.height, probe.width
    probe.close()
    out = np.empty((max(hi - lo, 0), H, W, 3), np.uint8)
    if hi <= lo:
        return out
    # GOP starts: I-VOPs (the first sample always starts one: a P-VOP there fails in the decoder)
    starts = [i for i in range(hi) if i == 0 or vop_coding_type(samples[i]) == 0]
    gops = [(a, b) for a, b in zip(starts, starts[1:] + [hi]) if b > lo]

    def run(g):
        a, b = g
        dec = Mp4vDecoder(config)
        try:
            for i in range(a, b):
                if i >= lo:
                    dec.decode(samples[i], out=out[i - lo])
                else:
                    dec.decode(samples[i])
        finally:
            dec.close()

    workers = max(1, min(int(threads or os.cpu_count() or 1), 16, len(gops)))
    if workers == 1:
        for g in gops:
            run(g)
    else:
        with ThreadPoolExecutor(workers) as pool:
            list(pool.map(run, gops))
    return out


MB_REC_BYTES = 32     # csrc/mp4v.h MbRec
JOB_DTYPE = np.dtype([("rec", "<u8"), ("coef", "<u8"), ("cur", "<u8"), ("ref", "<u8"), ("bgr", "<u8"),
                      ("coded", "<i4"), ("rounding", "<i4")])  # csrc/mp4v.h Job, 48 B


class Mp4vParser:
    """Host half of the split decode (mvp_mp4v_parse): entropy decoding, DC / AC and motion-vector
    prediction and inverse quantisation of one sample -> (records, coefficients, coded, rounding);
    the pixels are reconstructed on the device (mvp_mp4v_reconstruct)."""

    def __init__(self, config: bytes):
        import ctypes
        from . import _lib
        self._lib = _lib
        self._h = ctypes.c_void_p()
        w, h = ctypes.c_int(), ctypes.c_int()
        cfg = (ctypes.c_uint8 * max(1, len(config))).from_buffer_copy(config or b"\0")
        _lib.call("mvp_mp4v_create", cfg, len(config), ctypes.byref(self._h), ctypes.byref(w), ctypes.byref(h))
        self.width, self.height = w.value, h.value
        self.n_mb = ((self.width + 15) // 16) * ((self.height + 15) // 16)
        self._rec = np.empty(self.n_mb * MB_REC_BYTES, np.uint8)
        self._coef = np.empty(self.n_mb * 384, np.uint32)

    def parse(self, sample: bytes, rec_out: np.ndarray | None = None):
        """-> (records (n_mb * 32 uint8; rec_out when given) or None for a sample without a coded
        VOP, inverse-quantised coefficient entries (uint32, a view of this parser's scratch:
        copy before the next parse), coded (1 / 0 not coded / -1 no VOP), vop_rounding_type)."""
        import ctypes
        data = np.frombuffer(sample, np.uint8)
        rec = self._rec if rec_out is None else rec_out
        if rec.dtype != np.uint8 or rec.size < self.n_mb * MB_REC_BYTES or not rec.flags.c_contiguous:
            raise ValueError(f"rec_out must be a C-contiguous uint8 array of >= {self.n_mb * MB_REC_BYTES} bytes")
        n = ctypes.c_int64()
        vop = (ctypes.c_int * 2)()
        self._lib.call("mvp_mp4v_parse", self._h, data.ctypes.data, data.size, rec.ctypes.data, self.n_mb,
                       self._coef.ctypes.data, self._coef.size, ctypes.byref(n), vop)
        coded = int(vop[0])
        return (rec if coded == 1 else None, self._coef[:n.value], coded, int(vop[1]))

    def close(self):
        if self._h:
            self._lib.call("mvp_mp4v_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def decode_mp4v_device(config: bytes, samples, start=0, end=None, threads=None, device="cuda", stream=None,
                       timings: dict | None = None):
    """decode_mp4v with the pixels reconstructed on the GPU: frames [start:end) as a (n, H, W, 3)
    uint8 BGR tensor on `device`, bit-identical to decode_mp4v's host frames.

    The GOPs holding wanted frames are entropy-decoded on a host thread pool (mvp_mp4v_parse:
    one 32-B record per macroblock + the non-zero inverse-quantised coefficients, ~5-10 % of a
    BGR frame's bytes), copied to the device in one transfer, and reconstructed there by one
    mvp_mp4v_reconstruct launch per GOP position: every GOP is an independent slot with its own
    two pictures, so a launch runs one VOP of every GOP.  timings: filled with the host phases'
    seconds (parse, pack, launch; the launches are asynchronous)."""
    import time
    import torch
    from . import _lib
    samples = list(samples)
    if not config and samples:
        config = samples[0]
    keep = range(len(samples))[slice(start, end)]
    lo, hi = (keep.start, keep.stop) if len(keep) and keep.step == 1 else (0, 0)
    probe = Mp4vParser(config)
    H, W, n_mb = probe.height, probe.width, probe.n_mb
    probe.close()
    dev = torch.device(device)
    out = torch.empty((max(hi - lo, 0), H, W, 3), dtype=torch.uint8, device=dev)
    if hi <= lo:
        return out
    starts = [i for i in range(hi) if i == 0 or vop_coding_type(samples[i]) == 0]
    gops = [(a, b) for a, b in zip(starts, starts[1:] + [hi]) if b > lo]

    n_s = sum(b - a for a, b in gops)
    gop_base = np.concatenate([[0], np.cumsum([b - a for a, b in gops])]).astype(np.int64)
    rb = n_mb * MB_REC_BYTES
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    # records straight into one pinned buffer (torch caches pinned blocks across calls); each
    # GOP's records and coefficients go to the device on a copy stream as soon as it is parsed,
    # under the other GOPs' parsing
    rec_h = torch.empty(max(1, n_s * rb), dtype=torch.uint8, pin_memory=True)
    rec_np = rec_h.numpy()
    with torch.cuda.stream(s):
        rec_d = torch.empty(max(1, n_s * rb), dtype=torch.uint8, device=dev)
    copy_stream = torch.cuda.Stream(dev)
    copy_stream.wait_stream(s)                           # rec_d's allocation precedes the copies

    def parse(gi):
        """One GOP in native calls (mvp_mp4v_parse_many: the GIL is released for the whole GOP),
        then its H2D copies -> (its coefficients on the device, per-sample entry counts,
        per-sample [coded, rounding])."""
        import ctypes
        a, b = gops[gi]
        base, n = int(gop_base[gi]), b - a
        datas = [x if isinstance(x, bytes) else bytes(x) for x in samples[a:b]]
        ptrs = (ctypes.c_char_p * n)(*datas)
        sizes = np.array([len(x) for x in datas], np.uint64)
        ncoef = np.zeros(n, np.int64)
        vops = np.zeros((n, 2), np.int32)
        chunks, k = [], 0
        ps = Mp4vParser(config)
        try:
            while k < n:
                cap = n_mb * 384 + (n - k) * n_mb * 24
                buf = np.empty(cap, np.uint32)
                done = ctypes.c_int()
                _lib.call("mvp_mp4v_parse_many", ps._h, n - k, ctypes.addressof(ptrs) + 8 * k,
                          sizes.ctypes.data + 8 * k, rec_np[(base + k) * rb:].ctypes.data, buf.ctypes.data, cap,
                          ncoef.ctypes.data + 8 * k, vops.ctypes.data + 8 * k, ctypes.byref(done))
                chunks.append(buf[:int(ncoef[k:k + done.value].sum())])
                k += done.value
        finally:
            ps.close()
        cnt = int(ncoef.sum())
        coef_h = torch.empty(max(1, cnt), dtype=torch.int32, pin_memory=True)
        if cnt:
            np.concatenate(chunks, out=coef_h.numpy()[:cnt].view(np.uint32))
        with torch.cuda.stream(copy_stream):
            rec_d[base * rb:(base + n) * rb].copy_(rec_h[base * rb:(base + n) * rb], non_blocking=True)
            coef_d = coef_h.to(dev, non_blocking=True)
        coef_d.record_stream(s)                           # read by the reconstruction launches
        return coef_d, ncoef, vops

    t_parse = time.perf_counter()
    workers = max(1, min(int(threads or os.cpu_count() or 1), 16, len(gops)))
    if workers == 1:
        parsed = [parse(g) for g in range(len(gops))]
    else:
        with ThreadPoolExecutor(workers) as pool:
            parsed = list(pool.map(parse, range(len(gops))))
    t_pack = time.perf_counter()
    # per sample, in GOP order: coded flag, rounding, coefficient count
    coded = np.concatenate([v[:, 0] for _, _, v in parsed]).astype(np.int64)
    rnd = np.concatenate([v[:, 1] for _, _, v in parsed]).astype(np.int64)
    ncoef = [c for _, c, _ in parsed]
    coef_ptr = np.concatenate([d.data_ptr() + 4 * (np.cumsum(c) - c) for d, c, _ in parsed])
    nc = int(sum(int(c.sum()) for c in ncoef))
    gop_of = np.repeat(np.arange(len(gops)), [b - a for a, b in gops])
    step = np.arange(n_s) - gop_base[gop_of]
    frame = np.array([a for a, _ in gops], np.int64)[gop_of] + step
    # the host decoder's picture swap: a coded VOP writes the slot's other picture
    is_coded = (coded == 1).astype(np.int64)
    seen = np.zeros(n_s, np.int64)
    for g in range(len(gops)):
        sl = slice(int(gop_base[g]), int(gop_base[g + 1]))
        seen[sl] = np.cumsum(is_coded[sl])
    if (seen == 0).any():
        raise _lib.MvposeError(f"mp4v: sample {int(frame[np.argmax(seen == 0)])} repeats a frame before any was "
                               "decoded")
    cur_i = seen & 1
    pic_w, pic_h = 16 * ((W + 15) // 16), 16 * ((H + 15) // 16)
    pic_bytes = pic_w * pic_h * 3 // 2
    t_launch = time.perf_counter()
    with torch.cuda.stream(s):
        pics = torch.full((len(gops), 2, pic_bytes), 128, dtype=torch.uint8, device=dev)
        steps = int(step.max()) + 1
        # one job per sample; launch k runs the k-th VOP of every GOP that has one
        slot = pics.data_ptr() + gop_of * 2 * pic_bytes
        jl = np.zeros(n_s, JOB_DTYPE)
        jl["rec"] = rec_d.data_ptr() + np.arange(n_s, dtype=np.int64) * rb
        jl["coef"] = coef_ptr
        jl["cur"] = slot + cur_i * pic_bytes
        jl["ref"] = slot + (cur_i ^ 1) * pic_bytes
        jl["bgr"] = np.where(frame >= lo, out.data_ptr() + (frame - lo) * (H * W * 3), 0)
        jl["coded"] = is_coded
        jl["rounding"] = rnd
        order = np.lexsort((gop_of, step))                 # by step, then GOP
        n_jobs = np.bincount(step, minlength=steps)
        jobs_d = torch.from_numpy(jl[order].view(np.uint8).copy()).pin_memory().to(dev, non_blocking=True)
        s.wait_stream(copy_stream)
        first = np.concatenate([[0], np.cumsum(n_jobs)])
        for k in range(steps):
            _lib.call("mvp_mp4v_reconstruct", jobs_d.data_ptr() + int(first[k]) * JOB_DTYPE.itemsize, int(n_jobs[k]),
                      W, H, s.cuda_stream)
    if timings is not None:
        t_end = time.perf_counter()
        timings.update(parse=t_pack - t_parse, pack=t_launch - t_pack, launch=t_end - t_launch,
                       coef_entries=nc, gops=len(gops), samples=n_s)
    return out


def read_m4v(path, start=0, end=None, device=None):
    """A raw MPEG-4 Part 2 elementary stream (.m4v / .cmp)."""
    with open(path, "rb") as f:
        config, samples = split_vops(f.read())
    return _mp4v(config, samples, start, end, device)


class Mp4Info:
    def __init__(self, width, height, fps, config, samples):
        self.width, self.height, self.fps, self.config, self.samples = width, height, fps, config, samples

    def __len__(self):
        return len(self.samples)


def _boxes(buf, start, end):
    p = start
    while p + 8 <= end:
        size, kind = struct.unpack_from(">I4s", buf, p)
        hdr = 8
        if size == 1:
            size = struct.unpack_from(">Q", buf, p + 8)[0]
            hdr = 16
        elif size == 0:
            size = end - p
        if size < hdr or p + size > end:
            break
        yield kind, p + hdr, p + size
        p += size


def _descriptor(buf, p):
    """MPEG-4 descriptor at p -> (tag, payload start, payload end)."""
    tag = buf[p]
    p += 1
    size = 0
    for _ in range(4):
        b = buf[p]
        p += 1
        size = (size << 7) | (b & 0x7F)
        if not b & 0x80:
            break
    return tag, p, p + size


def _esds_config(buf, start, end):
    p = start + 4                                     # full box version / flags
    tag, p, e = _descriptor(buf, p)
    if tag != 0x03:
        return b""
    flags = buf[p + 2]
    p += 3
    if flags & 0x80:
        p += 2
    if flags & 0x40:
        p += 1 + buf[p]
    if flags & 0x20:
        p += 2
    while p < e:
        tag, q, qe = _descriptor(buf, p)
        if tag == 0x04:                               # DecoderConfigDescriptor
            oti = buf[q]
            if oti != 0x20:
                raise NotImplementedError(f"MP4 objectTypeIndication 0x{oti:02x} (only MPEG-4 Visual, 0x20)")
            r = q + 13
            while r < qe:
                t2, s2, e2 = _descriptor(buf, r)
                if t2 == 0x05:                        # DecoderSpecificInfo: the VOS / VOL headers
                    return bytes(buf[s2:e2])
                r = e2
        p = qe
    return b""


def parse_mp4(buf) -> Mp4Info:
    """The first video track of an ISO BMFF (MP4 / QuickTime) file: its 'mp4v' decoder config and
    the (offset, size) of every sample, from stsd / stsc / stco|co64 / stsz / stts / mdhd."""
    moov = next(((s, e) for k, s, e in _boxes(buf, 0, len(buf)) if k == b"moov"), None)
    if moov is None:
        raise ValueError("MP4: no moov box")
    for k, ts, te in _boxes(buf, *moov):
        if k != b"trak":
            continue
        mdia = next(((s, e) for kk, s, e in _boxes(buf, ts, te) if kk == b"mdia"), None)
        if mdia is None:
            continue
        parts = {kk: (s, e) for kk, s, e in _boxes(buf, *mdia)}
        if "hdlr".encode() not in parts or bytes(buf[parts[b"hdlr"][0] + 8:parts[b"hdlr"][0] + 12]) != b"vide":
            continue
        ms = parts[b"mdhd"][0]
        timescale = struct.unpack_from(">I", buf, ms + (20 if buf[ms] == 1 else 12))[0]
        minf = parts[b"minf"]
        stbl = next((s, e) for kk, s, e in _boxes(buf, *minf) if kk == b"stbl")
        t = {kk: (s, e) for kk, s, e in _boxes(buf, *stbl)}
        ss, se = t[b"stsd"]
        entry = next(_boxes(buf, ss + 8, se))
        kind, es, ee = entry
        if kind not in (b"mp4v", b"MP4V"):
            raise NotImplementedError(f"MP4 video codec {kind.decode('latin-1')!r}: only MPEG-4 Part 2 ('mp4v') "
                                      "can be decoded in this image (no H.264 / HEVC decoder)")
        width, height = struct.unpack_from(">HH", buf, es + 24)
        config = b""
        for kk, s, e in _boxes(buf, es + 78, ee):
            if kk == b"esds":
                config = _esds_config(buf, s, e)
        s, _ = t[b"stsz"]
        fixed, count = struct.unpack_from(">II", buf, s + 4)
        sizes = [fixed] * count if fixed else list(struct.unpack_from(f">{count}I", buf, s + 12))
        if b"stco" in t:
            s, _ = t[b"stco"]
            n = struct.unpack_from(">I", buf, s + 4)[0]
            chunks = list(struct.unpack_from(f">{n}I", buf, s + 8))
        else:
            s, _ = t[b"co64"]
            n = struct.unpack_from(">I", buf, s + 4)[0]
            chunks = list(struct.unpack_from(f">{n}Q", buf, s + 8))
        s, _ = t[b"stsc"]
        n = struct.unpack_from(">I", buf, s + 4)[0]
        stsc = [struct.unpack_from(">III", buf, s + 8 + 12 * i) for i in range(n)]
        samples, si = [], 0
        for ci, off in enumerate(chunks, start=1):
            per = next((spc for first, spc, _ in reversed(stsc) if first <= ci), 0)
            for _ in range(per):
                if si >= count:
                    break
                samples.append((off, sizes[si]))
                off += sizes[si]
                si += 1
        fps = 0.0
        if b"stts" in t and timescale:
            s, _ = t[b"stts"]
            n = struct.unpack_from(">I", buf, s + 4)[0]
            if n:
                delta = struct.unpack_from(">II", buf, s + 8)[1]
                fps = timescale / delta if delta else 0.0
        return Mp4Info(width, height, fps, config, samples)
    raise ValueError("MP4: no video track")


def read_mp4(path, start=0, end=None, device=None):
    """Frames [start:end) of an MP4 / QuickTime file with MPEG-4 Part 2 video -> (T, H, W, 3) BGR."""
    with open(path, "rb") as f:
        buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            info = parse_mp4(buf)
            return _mp4v(info.config, (bytes(buf[o:o + n]) for o, n in info.samples), start, end, device)
        finally:
            buf.close()


def write_avi(path, frames, fps=30.0, codec="mjpeg", quality=90):
    """Write (T, H, W, 3) uint8 BGR frames as an AVI (MJPEG or uncompressed 24-bit) with an
    idx1 index — for converting recordings and for the ingest tests."""
    frames = np.asarray(frames)
    if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[-1] != 3:
        raise ValueError("frames must be (T, H, W, 3) uint8")
    T, H, W, _ = frames.shape
    if codec == "mjpeg":
        from PIL import Image
        blobs = []
        for fr in frames:
            b = io.BytesIO()
            Image.fromarray(np.ascontiguousarray(fr[:, :, ::-1])).save(b, "JPEG", quality=int(quality))
            blobs.append(b.getvalue())
        cc, comp, bits = b"MJPG", struct.unpack("<I", b"MJPG")[0], 24
    elif codec == "rgb":
        stride = (W * 3 + 3) & ~3
        blobs = []
        for fr in frames:
            rows = np.zeros((H, stride), np.uint8)
            rows[:, :W * 3] = fr[::-1].reshape(H, W * 3)
            blobs.append(rows.tobytes())
        cc, comp, bits = b"\0\0\0\0", _BI_RGB, 24
    else:
        raise ValueError(f"codec {codec!r}")

    def chunk(cc4, data):
        return cc4 + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")

    def lst(kind, body):
        return b"LIST" + struct.pack("<I", len(body) + 4) + kind + body

    scale, rate = 1000, int(round(fps * 1000))
    maxb = max(len(b) for b in blobs) if blobs else 0
    avih = struct.pack("<IIIIIIIIII16x", int(1e6 / fps), 0, 0, 0x10, T, 0, 1, maxb, W, H)
    strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", cc, 0, 0, 0, 0, scale, rate, 0, T, maxb, 0xFFFFFFFF, 0,
                       0, 0, W, H)
    strf = struct.pack("<IiiHHIIiiII", 40, W, H, 1, bits, comp, (W * 3 + 3 & ~3) * H, 0, 0, 0, 0)
    hdrl = lst(b"hdrl", chunk(b"avih", avih) + lst(b"strl", chunk(b"strh", strh) + chunk(b"strf", strf)))
    movi_body, idx, off = b"", b"", 4
    tag = b"00dc" if codec == "mjpeg" else b"00db"
    for b in blobs:
        c = chunk(tag, b)
        idx += tag + struct.pack("<III", 0x10, off, len(b))
        movi_body += c
        off += len(c)
    body = b"AVI " + hdrl + lst(b"movi", movi_body) + chunk(b"idx1", idx)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)

