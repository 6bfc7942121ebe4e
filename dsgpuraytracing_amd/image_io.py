"""Minimal PNG / PFM writers for the output row (no third-party imaging libs).

PNG replaces lodepng::encode in PathTracer::save_image (pathtracer.cpp:649-674);
PFM stores the HDR sampleBuffer losslessly.
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
