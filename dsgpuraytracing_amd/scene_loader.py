"""Native host scene pipeline (include/ptgpu_scene.h) from Python.

load_dae() returns the flattened scene as a PTDUMP-style dict of numpy arrays
(the same layout oracle/_ref/ref_driver --mode dump writes), produced by the C++
restatement of ColladaParser + DynamicScene -> StaticScene + HalfedgeMesh +
buildBVH in libptgpu.so.
"""
from __future__ import annotations

import ctypes
import os
import tempfile
from typing import Dict, Optional

import numpy as np

from . import native, ptdump


def _bind(L):
    if getattr(L, "_scene_bound", False):
        return
    L.pt_host_scene_load.restype = ctypes.c_int32
    L.pt_host_scene_load.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                     ctypes.POINTER(ctypes.c_void_p)]
    L.pt_host_scene_view.restype = ctypes.c_int32
    L.pt_host_scene_view.argtypes = [ctypes.c_void_p, ctypes.POINTER(native.pt_scene),
                                     ctypes.POINTER(native.pt_camera)]
    L.pt_host_scene_dump.restype = ctypes.c_int32
    L.pt_host_scene_dump.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.pt_host_scene_free.restype = None
    L.pt_host_scene_free.argtypes = [ctypes.c_void_p]
    L._scene_bound = True


def dump_dae(path: str, width: int, height: int, out_path: str, cam_info: Optional[str] = None,
             envmap: Optional[str] = None) -> str:
    L = native.lib()
    _bind(L)
    h = ctypes.c_void_p()
    native.check(L.pt_host_scene_load(path.encode(), width, height, cam_info.encode() if cam_info else None,
                                      ctypes.byref(h)))
    try:
        if envmap:
            native.check(L.pt_host_scene_set_envmap(h, envmap.encode()))
        native.check(L.pt_host_scene_dump(h, out_path.encode()))
    finally:
        L.pt_host_scene_free(h)
    return out_path


def load_dae(path: str, width: int, height: int, cam_info: Optional[str] = None,
             envmap: Optional[str] = None) -> Dict[str, np.ndarray]:
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "scene.ptd")
        dump_dae(path, width, height, p, cam_info, envmap)
        return ptdump.read(p)


def load_exr(path: str) -> np.ndarray:
    """OpenEXR environment map -> float32 (h, w, 3), row 0 = first scanline,
    through the native reader (pt_host_load_exr: load_exr, main.cpp:30-67)."""
    L = native.lib()
    w, h = ctypes.c_int32(), ctypes.c_int32()
    p = ctypes.c_void_p()
    native.check(L.pt_host_load_exr(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)))
    try:
        n = w.value * h.value * 3
        arr = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(n,)).copy()
    finally:
        L.pt_host_free(p)
    return arr.reshape(h.value, w.value, 3)
