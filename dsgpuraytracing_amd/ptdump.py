"""Reader/writer for the PTDUMP01 tagged-array container (see csrc/ptdump.h).

Used for flattened scenes, ray batches and HDR images exchanged between the
host library, the oracle harness and the tests.
"""
from __future__ import annotations

import struct
from typing import Dict

import numpy as np

_MAGIC = b"PTDUMP01"
_DT = {"f8": np.float64, "f4": np.float32, "i4": np.int32, "i8": np.int64, "u4": np.uint32}


def read(path: str) -> Dict[str, np.ndarray]:
    out: Dict[str, np.ndarray] = {}
    with open(path, "rb") as f:
        if f.read(8) != _MAGIC:
            raise ValueError(f"{path}: not a PTDUMP01 file")
        while True:
            hdr = f.read(40)
            if len(hdr) != 40:
                raise ValueError(f"{path}: truncated record header")
            name = hdr[:24].split(b"\0", 1)[0].decode()
            dtype = hdr[24:32].split(b"\0", 1)[0].decode()
            (count,) = struct.unpack("<q", hdr[32:40])
            if name == "END":
                break
            dt = np.dtype(_DT[dtype])
            buf = f.read(count * dt.itemsize)
            if len(buf) != count * dt.itemsize:
                raise ValueError(f"{path}: truncated payload for {name}")
            out[name] = np.frombuffer(buf, dtype=dt).copy()
    return out


def write(path: str, arrays: Dict[str, np.ndarray]) -> None:
    inv = {np.dtype(v): k for k, v in _DT.items()}
    with open(path, "wb") as f:
        f.write(_MAGIC)
        for name, arr in arrays.items():
            a = np.ascontiguousarray(arr).reshape(-1)
            code = inv[a.dtype]
            f.write(name.encode()[:23].ljust(24, b"\0"))
            f.write(code.encode().ljust(8, b"\0"))
            f.write(struct.pack("<q", a.size))
            f.write(a.tobytes())
        f.write(b"END".ljust(24, b"\0") + b"i4".ljust(8, b"\0") + struct.pack("<q", 0))
