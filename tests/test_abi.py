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
