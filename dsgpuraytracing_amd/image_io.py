"""Minimal PNG / PFM / OpenEXR writers for the output row (no third-party
imaging libs).

PNG replaces lodepng::encode in PathTracer::save_image (pathtracer.cpp:649-674);
PFM stores the HDR sampleBuffer losslessly; OpenEXR (scanline, NONE or ZIP
compression, FLOAT or HALF channels B,G,R) writes environment maps the
reference's `-e` option (main.cpp:30-67, tinyexr) and our native loader
(csrc/exr_io.cpp) read.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def write_png(path: str, rgba: np.ndarray) -> None:
    """rgba: HxWx4 uint8, first row = top of the image."""
    h, w, c = rgba.shape
    assert c == 4 and rgba.dtype == np.uint8
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def write_pfm(path: str, hdr: np.ndarray) -> None:
    """hdr: HxWx3 float32 with row 0 = bottom (PFM's own row order)."""
    h, w, _ = hdr.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(hdr, dtype="<f4").tobytes())


def _exr_attr(name: str, typ: str, data: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def write_exr(path: str, rgb: np.ndarray, compression: str = "zip", half: bool = False) -> None:
    """rgb: HxWx3 float, row 0 = top (the OpenEXR and lat-long convention).
    compression "none" (1 scanline per block) or "zip" (16 scanlines, zlib
    over the predictor + interleave transform of the OpenEXR spec)."""
    h, w, _ = rgb.shape
    ptype = 1 if half else 2
    chans = b"".join(n + b"\0" + struct.pack("<iBBBBii", ptype, 0, 0, 0, 0, 1, 1) for n in (b"B", b"G", b"R")) + b"\0"
    comp = {"none": 0, "zip": 3}[compression]
    lines = 1 if comp == 0 else 16
    hdr = b"".join([
        _exr_attr("channels", "chlist", chans),
        _exr_attr("compression", "compression", bytes([comp])),
        _exr_attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1)),
        _exr_attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1)),
        _exr_attr("lineOrder", "lineOrder", bytes([0])),
        _exr_attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)),
        _exr_attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0)),
        _exr_attr("screenWindowWidth", "float", struct.pack("<f", 1.0)),
    ]) + b"\0"
    dt = np.dtype("<f2") if half else np.dtype("<f4")
    blocks = []
    for y0 in range(0, h, lines):
        y1 = min(h, y0 + lines)
        # per scanline: all B, then all G, then all R
        raw = b"".join(np.ascontiguousarray(rgb[y, :, c], dtype=dt).tobytes() for y in range(y0, y1) for c in (2, 1, 0))
        if comp == 3:
            b = np.frombuffer(raw, np.uint8)
            inter = np.concatenate([b[0::2], b[1::2]])          # interleave: even bytes then odd bytes
            pred = inter.astype(np.int16)
            pred[1:] = (inter[1:].astype(np.int16) - inter[:-1].astype(np.int16) + 128) & 0xFF  # predictor
            raw = zlib.compress(pred.astype(np.uint8).tobytes(), 6)
        blocks.append(struct.pack("<ii", y0, len(raw)) + raw)
    magic = struct.pack("<ii", 20000630, 2)
    start = len(magic) + len(hdr) + 8 * len(blocks)
    offs, o = [], start
    for b in blocks:
        offs.append(o)
        o += len(b)
    with open(path, "wb") as f:
        f.write(magic + hdr + struct.pack("<%dQ" % len(offs), *offs) + b"".join(blocks))
