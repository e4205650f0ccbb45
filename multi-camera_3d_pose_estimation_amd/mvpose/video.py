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

Every reader returns (T, H, W, 3) uint8 frames in the channel order cv2 returns them
(BGR), so the rest of the pipeline applies the reference's cvtColor(RGB2BGR) swap exactly
as for decoded video.  MPEG-4 / H.264 files raise NotImplementedError.  Decoded pixels
are libjpeg's (islow IDCT, fancy upsampling), which is what cv2.imread uses; cv2's
VideoCapture decodes MJPEG with FFmpeg's decoder instead, so MJPEG parity with the
reference is unpinned (no cv2 here to compare with).
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
                                          comp_cc.decode("latin-1"))
    return AviInfo(width, height, codec, bit_count, rate / scale if scale else 0.0, st["chunks"])


def _decode_jpeg(data: bytes) -> np.ndarray:
    from PIL import Image
    im = Image.open(io.BytesIO(data))
    rgb = np.asarray(im.convert("RGB"))
    return rgb[:, :, ::-1]             # BGR, as cv2 returns frames


def read_avi(path, start=0, end=None, threads=None) -> np.ndarray:
    """Frames [start:end) of an MJPEG / uncompressed AVI -> (T, H, W, 3) uint8 BGR."""
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


def read_recording(path, start=0, end=-1):
    """One camera's recording, sliced [start:end] with Python semantics (the reference's
    default [0, -1] drops the last frame) -> (T, H, W, 3) uint8 BGR (memory-mapped for .npy)."""
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
        return read_avi(p, start, end)
    raise NotImplementedError(
        f"{p}: no decoder for this container/codec in this image (MJPEG/uncompressed AVI, frame*.jpg "
        "directories and .npy stacks are supported; convert other videos to one of these)")


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

