"""ctypes binding of the C ABI in include/ptgpu.h (libptgpu.so).

The library is the product: there is no Python or CPU fallback for the render
path.  If the in-tree ``libptgpu.so`` is missing or fails to load, every entry
point raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint32, c_void_p

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libptgpu.so")

PT_OK = 0
PT_E_INVALID = -1
PT_E_HIP = -2
PT_E_NOSCENE = -3
PT_E_ALLOC = -4
PT_E_IO = -5
PT_LIGHT_ENVIRONMENT = 4
PT_FLAG_STATS = 1
PT_FLAG_REF_COUNTS = 2
PT_FLAG_PACKED = 4
PT_FLAG_PACKED16 = 8
PT_MAX_FRAMES = 8  # frames per pt_render_frames_device launch (include/ptgpu.h)

PRIM_SPHERE, PRIM_TRIANGLE = 0, 1
BSDF_DIFFUSE, BSDF_MIRROR, BSDF_REFRACTION, BSDF_GLASS, BSDF_EMISSION = range(5)
LIGHT_DIRECTIONAL, LIGHT_HEMISPHERE, LIGHT_POINT, LIGHT_AREA = range(4)


class NativeLibraryError(RuntimeError):
    pass


class PtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ptgpu error {code}: {msg}")
        self.code = code


class pt_bsdf(ctypes.Structure):
    _fields_ = [("type", c_int32), ("albedo", c_float * 3), ("transmittance", c_float * 3),
                ("emission", c_float * 3), ("ior", c_float), ("roughness", c_float)]


class pt_light(ctypes.Structure):
    _fields_ = [("type", c_int32), ("radiance", c_float * 3), ("position", c_double * 3),
                ("direction", c_double * 3), ("dim_x", c_double * 3), ("dim_y", c_double * 3),
                ("area", c_float)]


class pt_camera(ctypes.Structure):
    _fields_ = [("pos", c_double * 3), ("c2w", c_double * 9), ("screen_w", c_double),
                ("screen_h", c_double), ("screen_dist", c_double)]


class pt_bvh_node(ctypes.Structure):
    _fields_ = [("bb_min", c_double * 3), ("bb_max", c_double * 3), ("start", c_int64),
                ("range", c_int64), ("left", c_int64), ("right", c_int64)]


class pt_scene(ctypes.Structure):
    _fields_ = [("n_prims", c_int64), ("prim_type", POINTER(c_int32)), ("prim_bsdf", POINTER(c_int32)),
                ("prim_geom", POINTER(c_double)), ("prim_norm", POINTER(c_double)),
                ("n_nodes", c_int64), ("nodes", POINTER(pt_bvh_node)),
                ("n_bsdfs", c_int32), ("bsdfs", POINTER(pt_bsdf)),
                ("n_lights", c_int32), ("lights", POINTER(pt_light)),
                ("env_width", c_int32), ("env_height", c_int32), ("env_rgb", POINTER(c_float))]


class pt_params(ctypes.Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("spp", c_int32), ("max_depth", c_int32),
                ("ns_area_light", c_int32), ("seed", c_uint32), ("sample_base", c_uint32)]


class pt_tile(ctypes.Structure):
    _fields_ = [("x", c_int32), ("y", c_int32), ("w", c_int32), ("h", c_int32)]


class pt_stats(ctypes.Structure):
    _fields_ = [("pixels", c_int64), ("samples", c_int64), ("camera_rays", c_int64),
                ("bounce_rays", c_int64), ("shadow_rays", c_int64), ("node_visits", c_int64),
                ("tri_tests", c_int64), ("sphere_tests", c_int64), ("ext_hits", c_int64),
                ("last_ms", c_double), ("counters_valid", c_int32), ("grid_blocks", c_int32),
                ("blocks_per_cu", c_int32), ("wave_trav_steps", c_int64), ("wave_rounds", c_int64),
                ("culled_samples", c_int64), ("queue_atomics", c_int64),
                ("shade_clocks", c_int64), ("trav_clocks", c_int64),
                ("max_wave_clocks", c_int64), ("wave_wall_sum", c_int64), ("wave_wall_max", c_int64),
                ("leaf_steps", c_int64), ("hitshade_clocks", c_int64), ("resolve_ms", c_double),
                ("bvh_stack", c_int32), ("bvh_nodes", c_int64), ("section_clocks", c_int64 * 4),
                ("wave_span", c_int64 * 5), ("group_spp", c_int32), ("lane_iters", c_int64 * 4),
                ("deep_stack_steps", c_int64), ("partial_bytes", c_int64),
                ("footprint", c_int32 * 4), ("slot_latency_hist", c_int64 * 32), ("node_census", c_int64 * 8),
                ("frames_per_launch", c_int32), ("tile_zorder", c_int32)]


# Every symbol include/ptgpu.h and include/ptgpu_scene.h declare, with ctypes signatures.
_SIGS = {
    "pt_create": (c_int32, [c_int32, POINTER(c_void_p)]),
    "pt_destroy": (c_int32, [c_void_p]),
    "pt_upload_scene": (c_int32, [c_void_p, POINTER(pt_scene)]),
    "pt_upload_scene_lbvh": (c_int32, [c_void_p, POINTER(pt_scene)]),
    "pt_set_camera": (c_int32, [c_void_p, POINTER(pt_camera)]),
    "pt_set_params": (c_int32, [c_void_p, POINTER(pt_params)]),
    "pt_render_tiles": (c_int32, [c_void_p, POINTER(pt_tile), c_int32, c_void_p, c_uint32]),
    "pt_render_tiles_device": (c_int32, [c_void_p, POINTER(pt_tile), c_int32, c_void_p, c_void_p, c_uint32]),
    "pt_render_frames_device": (c_int32, [c_void_p, POINTER(pt_tile), c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                          c_uint32]),
    "pt_tile_submit": (c_int32, [c_void_p, POINTER(pt_tile), c_void_p, c_void_p]),
    "pt_tile_finish": (c_int32, [c_void_p]),
    "pt_intersect": (c_int32, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "pt_get_stats": (c_int32, [c_void_p, POINTER(pt_stats)]),
    "pt_get_launch_times": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, POINTER(c_int32)]),
    "pt_get_wave_trace": (c_int32, [c_void_p, c_void_p, c_int64, POINTER(c_int64)]),
    "pt_last_error": (c_char_p, []),
    "pt_to_color": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p]),
    "pt_to_color_check": (c_int64, [c_uint32, c_uint32]),
    "pt_env_search_check": (c_int64, [c_void_p, c_int32, c_int32, c_int64, c_void_p, c_void_p, POINTER(c_int64)]),
    # include/ptgpu_scene.h (bound with full types in scene_loader.py)
    "pt_host_scene_load": (c_int32, [c_char_p, c_int32, c_int32, c_char_p, POINTER(c_void_p)]),
    "pt_host_scene_view": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "pt_host_scene_dump": (c_int32, [c_void_p, c_char_p]),
    "pt_host_scene_free": (None, [c_void_p]),
    "pt_host_scene_set_envmap": (c_int32, [c_void_p, c_char_p]),
    "pt_host_load_exr": (c_int32, [c_char_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_void_p)]),
    "pt_host_free": (None, [c_void_p]),
    "pt_host_build_render_tree": (c_int32, [c_void_p, c_void_p, POINTER(c_int64), c_void_p]),
}

_lib = None


def _init_torch_hip_first():
    """PyTorch-ROCm wheels bundle their own HIP runtime beside the system one
    this library links (/opt/rocm).  In one process the two coexist only if
    torch's initialises first: after ours has opened the device, torch reports
    "No HIP GPUs are available".  So when torch is already imported, its HIP
    state is initialised before this library is loaded (a no-op without a GPU)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None:
        return
    try:
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:  # no GPU / CPU-only torch: nothing to order
        pass


def lib():
    """Load libptgpu.so (once).  Raises NativeLibraryError if it is absent.
    PT_LIB=<path> loads another build of the same library instead (A/B
    experiments, tools/ab.sh); it is never a fallback."""
    global _lib, LIB_PATH
    if _lib is not None:
        return _lib
    if os.environ.get("PT_LIB"):
        LIB_PATH = os.path.abspath(os.environ["PT_LIB"])
    _init_torch_hip_first()
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build it with `python -m dsgpuraytracing_amd.build` "
            "(or __graft_entry__.build()); the HIP path has no fallback")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIGS.items():
        if os.environ.get("PT_LIB") and not hasattr(L, name):
            continue  # (an older build in an A/B: it lacks a later diagnostics entry point)
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != PT_OK:
        raise PtError(rc, lib().pt_last_error().decode(errors="replace"))


def declared_symbols():
    return sorted(_SIGS)


# ---------------------------------------------------------------- scene payloads
class SceneArrays:
    """Host-side pt_scene: numpy arrays kept alive next to the ctypes struct.

    Built from a PTDUMP dict (oracle/_ref/ref_driver --mode dump, or the native
    loader's dump): primitives in BVH order, reference BVH topology, BSDF and
    light tables, camera.
    """

    def __init__(self, d):
        self.d = d
        self.prim_type = np.ascontiguousarray(d["prim_type"], dtype=np.int32)
        self.prim_bsdf = np.ascontiguousarray(d["prim_bsdf"], dtype=np.int32)
        self.prim_geom = np.ascontiguousarray(d["prim_geom"], dtype=np.float64)
        self.prim_norm = np.ascontiguousarray(d["prim_norm"], dtype=np.float64)
        nbb = d["node_bb"].reshape(-1, 6)
        ninfo = d["node_info"].reshape(-1, 4)
        nn = nbb.shape[0]
        # pt_bvh_node = 6 doubles + 4 int64 (80 B): one structured array, no per-node Python
        rec = np.zeros(nn, dtype=np.dtype([("bb", "<f8", 6), ("info", "<i8", 4)]))
        assert rec.dtype.itemsize == ctypes.sizeof(pt_bvh_node)
        rec["bb"] = nbb
        rec["info"] = ninfo
        self._node_rec = rec
        self.nodes = ctypes.cast(rec.ctypes.data, POINTER(pt_bvh_node)) if nn else (pt_bvh_node * 1)()
        bt = d["bsdf_type"]
        bp = d["bsdf_params"].reshape(-1, 12)
        self.bsdfs = (pt_bsdf * len(bt))()
        for i, t in enumerate(bt):
            b = self.bsdfs[i]
            b.type = int(t)
            b.albedo[:] = bp[i, 0:3].tolist()
            b.transmittance[:] = bp[i, 3:6].tolist()
            b.emission[:] = bp[i, 6:9].tolist()
            b.ior = float(bp[i, 9])
            b.roughness = float(bp[i, 10])
        lt = d["light_type"]
        lr = d["light_rad"].reshape(-1, 3)
        lg = d["light_geom"].reshape(-1, 12)
        la = d["light_area"]
        self.lights = (pt_light * max(1, len(lt)))()
        for i, t in enumerate(lt):
            L = self.lights[i]
            L.type = int(t)
            L.radiance[:] = lr[i].tolist()
            L.position[:] = lg[i, 0:3].tolist()
            L.direction[:] = lg[i, 3:6].tolist()
            L.dim_x[:] = lg[i, 6:9].tolist()
            L.dim_y[:] = lg[i, 9:12].tolist()
            L.area = float(la[i])
        self.scene = pt_scene(
            n_prims=len(self.prim_type),
            prim_type=self.prim_type.ctypes.data_as(POINTER(c_int32)),
            prim_bsdf=self.prim_bsdf.ctypes.data_as(POINTER(c_int32)),
            prim_geom=self.prim_geom.ctypes.data_as(POINTER(c_double)),
            prim_norm=self.prim_norm.ctypes.data_as(POINTER(c_double)),
            n_nodes=nn, nodes=self.nodes,
            n_bsdfs=len(bt), bsdfs=self.bsdfs,
            n_lights=len(lt), lights=self.lights)
        if "env_rgb" in d:  # EnvironmentLight map (light type 4)
            eh, ew = (int(v) for v in d["env_shape"])
            self.env_rgb = np.ascontiguousarray(d["env_rgb"], dtype=np.float32)
            assert self.env_rgb.size == ew * eh * 3
            self.scene.env_width, self.scene.env_height = ew, eh
            self.scene.env_rgb = self.env_rgb.ctypes.data_as(POINTER(c_float))
        cam = d["cam"]
        self.camera = pt_camera()
        self.camera.pos[:] = cam[0:3].tolist()
        self.camera.c2w[:] = cam[3:12].tolist()
        self.camera.screen_w = float(cam[12])
        self.camera.screen_h = float(cam[13])
        self.camera.screen_dist = float(cam[14])

    @property
    def n_prims(self) -> int:
        return len(self.prim_type)
