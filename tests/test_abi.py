"""The C ABI library: loads, exports every symbol the public headers declare,
and reports errors through return codes (no GPU needed for these)."""
import ctypes
import os
import re

import pytest

from dsgpuraytracing_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for f in os.listdir(inc):
        if f.endswith(".h"):
            txt = open(os.path.join(inc, f)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            syms |= set(re.findall(r"\b(pt_[a-z_0-9]+)\s*\(", txt))
    return syms


def test_library_exports_every_declared_symbol():
    L = native.lib()
    syms = header_symbols()
    assert syms, "no declarations found"
    for s in sorted(syms):
        assert hasattr(L, s), f"libptgpu.so does not export {s}"
    assert syms == set(native.declared_symbols()), "ctypes signatures out of sync with the headers"


def test_invalid_arguments_return_codes():
    L = native.lib()
    assert L.pt_set_params(None, None) == native.PT_E_INVALID
    assert b"NULL" in L.pt_last_error()
    assert L.pt_get_stats(None, None) == native.PT_E_INVALID
    assert L.pt_create(0, None) == native.PT_E_INVALID
    assert L.pt_destroy(None) == native.PT_OK


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    rc = native.lib().pt_create(0, ctypes.byref(h))
    assert rc in (native.PT_E_HIP, native.PT_E_INVALID)
    assert native.lib().pt_last_error()


def test_struct_layouts_match_header():
    # sizes of the C structs as compiled into the library's ABI (x86-64 SysV)
    assert ctypes.sizeof(native.pt_bsdf) == 4 + 9 * 4 + 8
    assert ctypes.sizeof(native.pt_light) == 4 + 12 + 4 * 24 + 4 + 4  # trailing padding to 8
    assert ctypes.sizeof(native.pt_camera) == 15 * 8
    assert ctypes.sizeof(native.pt_bvh_node) == 6 * 8 + 4 * 8
    assert ctypes.sizeof(native.pt_params) == 28  # + sample_base
    assert ctypes.sizeof(native.pt_tile) == 16


def _fastdiv_init(d):
    """pt_fastdiv_init (csrc/pt_device.h), restated."""
    l = 0
    while (1 << l) < d:
        l += 1
    if (1 << l) == d:
        return 0, l
    return ((1 << (31 + l)) + d - 1) // d, l - 1


def _fastdiv(u, m, sh):
    return (u * m >> 32) >> sh if m else u >> sh


def test_fastdiv_exact():
    """The kernel's unit -> block division (pt_fastdiv: multiply-high and
    shift) equals integer division for every divisor up to 4096 over u < 2^31:
    exhaustively for small u, at every multiple of d and its neighbours near
    the top of the range, and at random points."""
    import numpy as np
    rng = np.random.default_rng(5)
    top = (1 << 31) - 1
    for d in list(range(1, 4097)) + [65535, 65536, 100003, (1 << 20) + 1]:
        m, sh = _fastdiv_init(d)
        assert m < (1 << 32)
        us = list(range(0, 2000)) + [top, top - 1] + [int(x) for x in rng.integers(0, top, 200)]
        k = top // d
        us += [k * d - 1, k * d, min(top, k * d + d - 1), (k - 1) * d, (k - 1) * d - 1]
        for u in us:
            if 0 <= u <= top:
                assert _fastdiv(u, m, sh) == u // d, (d, u)
