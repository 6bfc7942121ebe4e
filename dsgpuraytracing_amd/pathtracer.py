"""Host-side mirror of the reference's PathTracer interface over the HIP path.

Reference: class PathTracer (src/pathtracer.h:55-272, src/pathtracer.cpp).
Same names, argument meaning and state machine for the part of the interface
that drives the hot path:

  PathTracer(ns_aa, max_ray_depth, ns_area_light, ns_diff, ns_glsy, ns_refr,
             num_threads, envmap)                       pathtracer.cpp:30-66
  set_scene / set_camera / set_frame_size               pathtracer.cpp:76-122
  start_raytracing  (all tiles of the 32x32 FIFO)       pathtracer.cpp:192-221
  raytrace_tile(tile_x, tile_y, tile_w, tile_h)         pathtracer.cpp:585-611
  raytrace_pixel(x, y)                                  pathtracer.cpp:555-583
  sampleBuffer (HDR, float32 HxWx3, row 0 = bottom)     image.h:79-205
  frameBuffer  (RGBA8 after toColor)                    image.h:174-189
  save_image(path)                                      pathtracer.cpp:649-674

Every pixel is computed by libptgpu.so on the GPU; nothing here falls back to
the CPU.  `num_threads` is accepted for interface parity and ignored (the GPU
schedules itself).  Randomness comes from the counter stream keyed by
(seed, pixel, sample) instead of std::rand() (see csrc/pt_rng.h).
"""
from __future__ import annotations

import ctypes
import enum
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import native, ptdump
from .native import check, lib

TILE = 32  # imageTileSize (pathtracer.cpp:57)


def _flags(stats) -> int:
    """stats=True: counters of the launch itself; stats="ref": counters of the
    reference's binary BVH (PT_FLAG_REF_COUNTS, SURVEY.md §8(d) cost model)."""
    if stats == "ref":
        return native.PT_FLAG_REF_COUNTS
    return native.PT_FLAG_STATS if stats else 0


class Device:
    """One pt_ctx on one GPU (CUDAPathTracer's device state, setup.h:90-148)."""

    def __init__(self, device: int = 0):
        self._lib = lib()
        h = ctypes.c_void_p()
        check(self._lib.pt_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device
        self._scene_keepalive = None

    def close(self):
        if self.handle:
            self._lib.pt_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    def upload_scene(self, scene: "Scene", gpu_bvh: bool = False):
        """gpu_bvh: build a linear BVH on the device (pt_upload_scene_lbvh, the
        reference's PARALLEL_BUILD_BVH path) instead of using the scene's BVH."""
        fn = self._lib.pt_upload_scene_lbvh if gpu_bvh else self._lib.pt_upload_scene
        check(fn(self.handle, ctypes.byref(scene.arrays.scene)))
        self._scene_keepalive = scene

    def set_camera(self, cam: native.pt_camera):
        check(self._lib.pt_set_camera(self.handle, ctypes.byref(cam)))

    def set_params(self, width, height, spp, max_depth, ns_area_light, seed, sample_base=0):
        """sample_base: first sample index of this pass (pt_params.sample_base)."""
        p = native.pt_params(width=width, height=height, spp=spp, max_depth=max_depth,
                             ns_area_light=ns_area_light, seed=seed & 0xFFFFFFFF, sample_base=sample_base)
        check(self._lib.pt_set_params(self.handle, ctypes.byref(p)))
        self._frame = (int(height), int(width))

    @staticmethod
    def _tiles(tiles: Sequence[Tuple[int, int, int, int]]):
        """pt_tile[] view of the tile list (an int32 (n, 4) array; the caller
        keeps it alive for the duration of the call)."""
        if isinstance(tiles, np.ndarray) and tiles.dtype == np.int32 and tiles.flags.c_contiguous:
            arr = tiles.reshape(-1, 4)
        else:
            arr = np.ascontiguousarray(np.asarray(tiles, dtype=np.int32).reshape(-1, 4))
        return arr, arr.ctypes.data_as(ctypes.POINTER(native.pt_tile))

    def _check_frame(self, arr: np.ndarray, channels: int, dtype, what: str):
        """The native side writes (x + y*W)*channels elements of `arr` for the
        frame of the last set_params: anything smaller is refused here."""
        hw = getattr(self, "_frame", None)
        if hw is None:  # no frame yet: the native call refuses to render (PT_E_NOSCENE)
            return
        if arr.dtype != dtype or not arr.flags.c_contiguous or arr.shape != (hw[0], hw[1], channels):
            raise ValueError(f"{what}: need a C-contiguous {np.dtype(dtype).name} array of shape "
                             f"{(hw[0], hw[1], channels)}, got {arr.dtype} {arr.shape}")

    def render_tiles(self, tiles, out: np.ndarray, stats: bool = False):
        self._check_frame(out, 3, np.float32, "render_tiles")
        keep, arr = self._tiles(tiles)
        flags = _flags(stats)
        check(self._lib.pt_render_tiles(self.handle, arr, len(keep), out.ctypes.data, flags))

    def render_tiles_device(self, tiles, out_ptr: int, stream: int = 0, stats: bool = False, packed: bool = False,
                            out_floats: Optional[int] = None):
        """packed=True (or 32): out_ptr holds len(tiles)*32*32*3 floats, tile
        i's pixel (x, y) at [(i*1024 + (y-ty)*32 + (x-tx))*3] (PT_FLAG_PACKED);
        packed=16: 16x16 slots (PT_FLAG_PACKED16, tiles <= 16x16); else a
        whole H x W x 3 frame.  out_floats: the buffer's size in floats, checked
        against what the layout writes (the library sees only a pointer)."""
        keep, arr = self._tiles(tiles)
        if out_floats is not None:
            if getattr(self, "_frame", None) is None:
                raise ValueError("render_tiles_device: set_params first")
            need = len(keep) * _slot(packed) ** 2 * 3 if packed else self._frame[0] * self._frame[1] * 3
            if out_floats < need:
                raise ValueError(f"render_tiles_device: output holds {out_floats} floats, the "
                                 f"{'packed' if packed else 'frame'} layout writes {need}")
        flags = _flags(stats) | _packed_flag(packed)
        check(self._lib.pt_render_tiles_device(self.handle, arr, len(keep), ctypes.c_void_p(out_ptr),
                                               ctypes.c_void_p(stream or None), flags))

    def render_frames_device(self, tiles, out_ptrs, seeds, stream: int = 0, packed: bool = False,
                             out_floats: Optional[int] = None):
        """pt_render_frames_device: len(seeds) (1..8) frames of the same tiles in
        one launch, frame f keyed by seeds[f] into out_ptrs[f] (each laid out as
        render_tiles_device's out_ptr); every image equals its own
        render_tiles_device call with that seed."""
        n = len(seeds)
        if n != len(out_ptrs) or not 1 <= n <= native.PT_MAX_FRAMES:
            raise ValueError(f"render_frames_device: 1..{native.PT_MAX_FRAMES} frames, one output each")
        keep, arr = self._tiles(tiles)
        if out_floats is not None:
            if getattr(self, "_frame", None) is None:
                raise ValueError("render_frames_device: set_params first")
            need = len(keep) * _slot(packed) ** 2 * 3 if packed else self._frame[0] * self._frame[1] * 3
            if out_floats < need:
                raise ValueError(f"render_frames_device: outputs hold {out_floats} floats, the "
                                 f"{'packed' if packed else 'frame'} layout writes {need}")
        sd = (ctypes.c_uint32 * n)(*[int(v) & 0xFFFFFFFF for v in seeds])
        op = (ctypes.c_void_p * n)(*[int(v) for v in out_ptrs])
        flags = _packed_flag(packed)
        check(self._lib.pt_render_frames_device(self.handle, arr, len(keep), n, sd, op,
                                                ctypes.c_void_p(stream or None), flags))

    def submit_tile(self, tile, hdr: np.ndarray, rgba: Optional[np.ndarray] = None):
        """pt_tile_submit: queue one tile; its pixels land in `hdr` ((H, W, 3)
        float32) and, toColor'd, in `rgba` ((H, W, 4) uint8) when its batch
        completes.  Both arrays must stay alive until finish_tiles() returns
        (whatever it returns: it waits for every launched batch first).  The
        completion thread writes them long after this call, so their shapes
        are checked against the frame of the last set_params here."""
        self._check_frame(hdr, 3, np.float32, "submit_tile (hdr)")
        if rgba is not None:
            self._check_frame(rgba, 4, np.uint8, "submit_tile (rgba)")
        t = native.pt_tile(*[int(v) for v in tile])
        check(self._lib.pt_tile_submit(self.handle, ctypes.byref(t), hdr.ctypes.data,
                                       None if rgba is None else rgba.ctypes.data))

    def finish_tiles(self):
        """pt_tile_finish: render what is queued, wait for every submitted tile."""
        check(self._lib.pt_tile_finish(self.handle))

    def intersect(self, o, d, max_t):
        o = np.ascontiguousarray(o, np.float64)
        d = np.ascontiguousarray(d, np.float64)
        max_t = np.ascontiguousarray(max_t, np.float64)
        n = len(max_t)
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.int32)
        anyh = np.zeros(n, np.int32)
        check(self._lib.pt_intersect(self.handle, n, o.ctypes.data, d.ctypes.data, max_t.ctypes.data,
                                     hit.ctypes.data, t.ctypes.data, prim.ctypes.data, anyh.ctypes.data))
        return hit, t, prim, anyh

    def stats(self) -> dict:
        s = native.pt_stats()
        check(self._lib.pt_get_stats(self.handle, ctypes.byref(s)))
        out = {k: getattr(s, k) for k, _ in native.pt_stats._fields_}
        out["section_clocks"] = list(s.section_clocks)
        out["slot_latency_hist"] = list(s.slot_latency_hist)
        out["wave_span"] = list(s.wave_span)
        out["lane_iters"] = list(s.lane_iters)
        out["footprint"] = list(s.footprint)
        out["node_census"] = list(s.node_census)
        out["frames_per_launch"] = int(s.frames_per_launch)
        out["tile_zorder"] = int(s.tile_zorder)
        return out

    def launch_times(self, n: int = 256):
        """(kernel_ms, resolve_ms) arrays of the last <= n renders, oldest
        first, from HIP events recorded around each launch on its stream
        (pt_get_launch_times; waits for them)."""
        k = np.zeros(n, np.float32)
        r = np.zeros(n, np.float32)
        got = ctypes.c_int32(0)
        check(self._lib.pt_get_launch_times(self.handle, k.ctypes.data, r.ctypes.data, n, ctypes.byref(got)))
        return k[:got.value].copy(), r[:got.value].copy()

    def wave_trace(self) -> np.ndarray:
        """Per-wave records of the last stats launch (pt_get_wave_trace):
        int64 (waves, 11) = start, first empty-queue time (-1: never), end,
        (XCC id << 32 | HW_ID), camera samples started, sum and max of the
        work-slot latencies (wall-clock ticks, 100 MHz), per-ray maxima of
        traversal iterations stepped (<< 32) | idle, and of traversal phases,
        traversal iterations and shading rounds after the queue drained."""
        n = ctypes.c_int64(0)
        check(self._lib.pt_get_wave_trace(self.handle, None, 0, ctypes.byref(n)))
        buf = np.zeros((n.value, 11), np.int64)
        check(self._lib.pt_get_wave_trace(self.handle, buf.ctypes.data, buf.size, ctypes.byref(n)))
        return buf


class Scene:
    """A flattened scene (what BVHAccel + the lights hand to the GPU seam)."""

    def __init__(self, arrays: native.SceneArrays):
        self.arrays = arrays

    @classmethod
    def from_dump(cls, path: str) -> "Scene":
        return cls(native.SceneArrays(ptdump.read(path)))

    @classmethod
    def from_dae(cls, path: str, width: int, height: int, cam_info: Optional[str] = None,
                 envmap: Optional[str] = None) -> "Scene":
        """envmap: OpenEXR lat-long map for the EnvironmentLight (the reference's -e)."""
        from . import scene_loader
        return cls(native.SceneArrays(scene_loader.load_dae(path, width, height, cam_info, envmap)))

    @property
    def camera(self) -> native.pt_camera:
        return self.arrays.camera


class State(enum.IntEnum):
    INIT = 0
    READY = 1
    VISUALIZE = 2
    RENDERING = 3
    DONE = 4


def _slot(packed) -> int:
    """Packed slot edge of a `packed` argument: True / 32 -> 32, 16 -> 16."""
    return 16 if packed == 16 else 32


def _packed_flag(packed) -> int:
    if not packed:
        return 0
    return native.PT_FLAG_PACKED16 if _slot(packed) == 16 else native.PT_FLAG_PACKED


def tile_fifo(w: int, h: int, tile: int = TILE) -> List[Tuple[int, int, int, int]]:
    """The reference's row-major tile work queue (pathtracer.cpp:209-214)."""
    return [(x, y, tile, tile) for y in range(0, h, tile) for x in range(0, w, tile)]


def to_color(hdr: np.ndarray) -> np.ndarray:
    """HDRImageBuffer::toColor (image.h:174-189) + Color -> RGBA8
    (ImageBuffer::update_pixel, image.h:49-58) of a whole (H, W, 3) float32
    buffer, through libptgpu.so's pt_to_color (the reference's powf
    arithmetic, bit-exact: tests/test_output.py).  Returns (H, W, 4) uint8."""
    hdr = np.ascontiguousarray(hdr, dtype=np.float32)
    h, w = hdr.shape[:2]
    frame = np.zeros((h, w), np.uint32)
    native.check(native.lib().pt_to_color(hdr.ctypes.data, w, h, 0, 0, w, h, frame.ctypes.data))
    return frame.view(np.uint8).reshape(h, w, 4)


class PathTracer:
    def __init__(self, ns_aa: int = 1, max_ray_depth: int = 4, ns_area_light: int = 1, ns_diff: int = 1,
                 ns_glsy: int = 1, ns_refr: int = 1, num_threads: int = 1, envmap=None, device: int = 0,
                 seed: int = 1, gpu_bvh: bool = False):
        # envmap: an OpenEXR path or a float (h, w, 3) lat-long array; like the
        # reference (pathtracer.cpp:42-46, 88-90) it becomes an EnvironmentLight
        # appended to the scene's lights in set_scene.
        if isinstance(envmap, str):
            from . import scene_loader
            envmap = scene_loader.load_exr(envmap)
        self.envmap = None if envmap is None else np.ascontiguousarray(envmap, dtype=np.float32)
        self.state = State.INIT
        self.ns_aa = int(ns_aa)
        self.max_ray_depth = int(max_ray_depth)
        self.ns_area_light = int(ns_area_light)
        self.ns_diff, self.ns_glsy, self.ns_refr = ns_diff, ns_diff, ns_refr  # pathtracer.cpp:38-40 (sic)
        self.numWorkerThreads = int(num_threads)
        self.imageTileSize = TILE
        self.seed = int(seed)
        self.scene: Optional[Scene] = None
        self.camera: Optional[native.pt_camera] = None
        self.sampleBuffer = np.zeros((0, 0, 3), np.float32)
        self.frameBuffer = np.zeros((0, 0, 4), np.uint8)
        self._device_index = device
        self.gpu_bvh = bool(gpu_bvh)  # build the BVH on the GPU (PARALLEL_BUILD_BVH, setup.cu:188-189)
        self._dev: Optional[Device] = None
        self.last_stats: dict = {}

    # ---- configuration (pathtracer.cpp:76-127)
    def _device(self) -> Device:
        if self._dev is None:
            self._dev = Device(self._device_index)
        return self._dev

    def has_valid_configuration(self) -> bool:
        return self.scene is not None and self.camera is not None and self.sampleBuffer.size > 0

    def set_scene(self, scene: Scene):
        if self.state != State.INIT:
            return
        if self.envmap is not None and "env_rgb" not in scene.arrays.d:
            d = dict(scene.arrays.d)
            h, w, _ = self.envmap.shape
            d["light_type"] = np.append(d["light_type"], np.int32(native.PT_LIGHT_ENVIRONMENT)).astype(np.int32)
            d["light_rad"] = np.append(d["light_rad"], np.zeros(3, np.float32))
            d["light_geom"] = np.append(d["light_geom"], np.zeros(12))
            d["light_area"] = np.append(d["light_area"], np.float32(0))
            d["env_shape"] = np.array([h, w], np.int64)
            d["env_rgb"] = self.envmap.reshape(-1)
            scene = Scene(native.SceneArrays(d))
        self.scene = scene
        self._device().upload_scene(scene, gpu_bvh=self.gpu_bvh)
        if self.has_valid_configuration():
            self.state = State.READY

    def set_camera(self, camera: native.pt_camera):
        self.camera = camera
        self._device().set_camera(camera)
        if self.has_valid_configuration():
            self.state = State.READY

    def set_frame_size(self, width: int, height: int):
        self.sampleBuffer = np.zeros((height, width, 3), np.float32)
        self.frameBuffer = np.zeros((height, width, 4), np.uint8)
        if self.has_valid_configuration():
            self.state = State.READY

    def clear(self):
        if self.state != State.READY:
            return
        self.scene = None
        self.camera = None
        self.sampleBuffer = np.zeros((0, 0, 3), np.float32)
        self.frameBuffer = np.zeros((0, 0, 4), np.uint8)
        self.state = State.INIT

    # ---- rendering
    def _params(self):
        h, w = self.sampleBuffer.shape[:2]
        self._device().set_params(w, h, self.ns_aa, self.max_ray_depth, self.ns_area_light, self.seed)

    def raytrace_tile(self, tile_x: int, tile_y: int, tile_w: int, tile_h: int, stats: bool = False):
        """Drop-in for PathTracer::raytrace_tile: HDR for the tile, then toColor."""
        self.render_tiles([(tile_x, tile_y, tile_w, tile_h)], stats=stats)

    def render_tiles(self, tiles: Iterable[Tuple[int, int, int, int]], stats: bool = False):
        if not self.has_valid_configuration():
            raise RuntimeError("PathTracer is not configured (scene, camera, frame size)")
        tiles = list(tiles)
        self._params()
        dev = self._device()
        dev.render_tiles(tiles, self.sampleBuffer, stats=stats)
        self.last_stats = dev.stats()
        h, w = self.sampleBuffer.shape[:2]
        for (x, y, tw, th) in tiles:
            x1, y1 = min(x + tw, w), min(y + th, h)
            self.frameBuffer[y:y1, x:x1] = to_color(self.sampleBuffer[y:y1, x:x1])

    def render_tile_workers(self, num_threads: Optional[int] = None, asynchronous: bool = True,
                            tiles: Optional[Sequence[Tuple[int, int, int, int]]] = None):
        """The reference's tile workers (start_raytracing + worker_thread,
        pathtracer.cpp:192-221, 613-637): `num_threads` threads pop tiles from
        the 32x32 FIFO and call raytrace_tile on each, through ONE context
        (calls serialised by a lock, as INTEGRATION.md's adapter does).
        asynchronous=True: raytrace_tile is pt_tile_submit (tiles batched into
        launches, each completed into sampleBuffer/frameBuffer by the context's
        completion thread; the last worker's pt_tile_finish waits for all);
        asynchronous=False: one synchronous pt_render_tiles launch per tile."""
        import queue
        import threading
        if not self.has_valid_configuration():
            raise RuntimeError("PathTracer is not configured (scene, camera, frame size)")
        h, w = self.sampleBuffer.shape[:2]
        self._params()
        dev = self._device()
        work = queue.Queue()
        for t in (tile_fifo(w, h) if tiles is None else tiles):
            work.put(t)
        lock = threading.Lock()
        errors = []

        def worker():
            try:
                while True:
                    try:
                        t = work.get_nowait()
                    except queue.Empty:
                        return
                    if asynchronous:
                        with lock:
                            dev.submit_tile(t, self.sampleBuffer, self.frameBuffer)
                    else:
                        with lock:
                            dev.render_tiles([t], self.sampleBuffer)
                        x1, y1 = min(t[0] + t[2], w), min(t[1] + t[3], h)
                        self.frameBuffer[t[1]:y1, t[0]:x1] = to_color(self.sampleBuffer[t[1]:y1, t[0]:x1])
            except Exception as e:  # pragma: no cover - surfaced below
                errors.append(e)

        ths = [threading.Thread(target=worker) for _ in range(num_threads or self.numWorkerThreads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if asynchronous:
            dev.finish_tiles()
        if errors:
            raise errors[0]

    def raytrace_pixel(self, x: int, y: int) -> np.ndarray:
        self.raytrace_tile(x, y, 1, 1)
        return self.sampleBuffer[y, x].copy()

    def start_raytracing(self, stats: bool = False):
        """Whole frame: every tile of the FIFO in one batched launch."""
        if self.state != State.READY:
            return
        self.state = State.RENDERING
        self.sampleBuffer[...] = 0
        self.frameBuffer[...] = 0
        h, w = self.sampleBuffer.shape[:2]
        self.render_tiles(tile_fifo(w, h), stats=stats)
        self.state = State.DONE

    def stop(self):
        if self.state in (State.RENDERING, State.DONE):
            self.state = State.READY

    def save_image(self, path: str):
        """Writes frameBuffer flipped vertically (pathtracer.cpp:662-672) as PNG."""
        from .image_io import write_png
        write_png(path, self.frameBuffer[::-1])
