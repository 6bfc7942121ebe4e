"""Test-side access to the oracle (oracle/restate.cpp, oracle/_ref).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module; the product (dsgpuraytracing_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
RESTATE_SO = os.path.join(ORACLE, "_build", "librestate.so")
REF_DRIVER = os.path.join(ORACLE, "_ref", "ref_driver")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def build_restatement() -> str:
    src = os.path.join(ORACLE, "restate.cpp")
    if not os.path.exists(RESTATE_SO) or os.path.getmtime(RESTATE_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-C", ORACLE, "-s"], check=True)
    return RESTATE_SO


class Restatement:
    def __init__(self):
        self.lib = ctypes.CDLL(build_restatement())
        self.lib.rs_render.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 5 + [ctypes.c_uint32] + \
            [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.rs_render.restype = ctypes.c_int
        self.lib.rs_render_strided.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 5 + [ctypes.c_uint32] + \
            [ctypes.c_int] * 5 + [ctypes.c_void_p] * 3
        self.lib.rs_render_strided.restype = ctypes.c_int
        self.lib.rs_intersect.argtypes = [ctypes.c_char_p, ctypes.c_int64] + [ctypes.c_void_p] * 8
        self.lib.rs_intersect.restype = ctypes.c_int
        self.lib.rs_pixel_samples.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 5 + [ctypes.c_uint32, ctypes.c_int] + \
            [ctypes.c_void_p] * 3
        self.lib.rs_pixel_samples.restype = ctypes.c_int
        self.lib.rs_rng_draw.argtypes = [ctypes.c_uint32] * 4
        self.lib.rs_rng_draw.restype = ctypes.c_double

    def render(self, scene_path, w, h, spp, depth=4, ns_area_light=1, seed=1, rng_mode=0, threads=1,
               tile_begin=0, tile_end=-1):
        out = np.zeros((h, w, 3), np.float32)
        st = np.zeros(5, np.int64)
        rc = self.lib.rs_render(scene_path.encode(), w, h, spp, depth, ns_area_light, seed, rng_mode, threads,
                                tile_begin, tile_end, out.ctypes.data, st.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"rs_render failed on {scene_path}")
        return out, st

    def render_strided(self, scene_path, w, h, spp, depth=4, ns_area_light=1, seed=1, rng_mode=0, threads=1,
                       tile_begin=0, tile_end=-1, tile_stride=1):
        """Tiles tile_begin, +stride, ... < tile_end; returns (hdr, stats, render seconds)."""
        out = np.zeros((h, w, 3), np.float32)
        st = np.zeros(5, np.int64)
        secs = ctypes.c_double(0.0)
        rc = self.lib.rs_render_strided(scene_path.encode(), w, h, spp, depth, ns_area_light, seed, rng_mode,
                                        threads, tile_begin, tile_end, tile_stride, out.ctypes.data,
                                        st.ctypes.data, ctypes.byref(secs))
        if rc != 0:
            raise RuntimeError(f"rs_render_strided failed on {scene_path}")
        return out, st, secs.value

    def pixel_samples(self, scene_path, w, h, spp, xs, ys, depth=4, ns_area_light=1, seed=1):
        """(len(xs), spp, 3) radiance of every sample of the listed pixels (counter RNG)."""
        xs = np.ascontiguousarray(xs, np.int32)
        ys = np.ascontiguousarray(ys, np.int32)
        out = np.zeros((len(xs), spp, 3), np.float32)
        rc = self.lib.rs_pixel_samples(scene_path.encode(), w, h, spp, depth, ns_area_light, seed, len(xs),
                                       xs.ctypes.data, ys.ctypes.data, out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"rs_pixel_samples failed on {scene_path}")
        return out

    def intersect(self, scene_path, o, d, maxt):
        n = len(maxt)
        o = np.ascontiguousarray(o, np.float64)
        d = np.ascontiguousarray(d, np.float64)
        maxt = np.ascontiguousarray(maxt, np.float64)
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float64)
        prim = np.zeros(n, np.int32)
        nrm = np.zeros(3 * n, np.float64)
        anyh = np.zeros(n, np.int32)
        rc = self.lib.rs_intersect(scene_path.encode(), n, o.ctypes.data, d.ctypes.data, maxt.ctypes.data,
                                   hit.ctypes.data, t.ctypes.data, prim.ctypes.data, nrm.ctypes.data,
                                   anyh.ctypes.data)
        if rc != 0:
            raise RuntimeError("rs_intersect failed")
        return hit, t, prim, nrm.reshape(-1, 3), anyh

    def rng_draw(self, seed, pixel, sample, k):
        return self.lib.rs_rng_draw(seed, pixel, sample, k)


def golden(name: str) -> str:
    return os.path.join(GOLDEN, name)


def box_downsample(img: np.ndarray, k: int = 8) -> np.ndarray:
    """k x k box average of an (H, W, 3) image (H, W multiples of k)."""
    h, w, c = img.shape
    return img.astype(np.float64).reshape(h // k, k, w // k, k, c).mean(axis=(1, 3))


def downsampled_rel_l2(img: np.ndarray, ref: np.ndarray, k: int = 8) -> float:
    """SURVEY.md §8(c) criterion 3, last clause: ||D(img) - D(ref)|| / ||D(ref)||
    over every channel of the k x k box-downsampled images."""
    a, b = box_downsample(img, k), box_downsample(ref, k)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def statistical_report(img: np.ndarray, r1: np.ndarray, r2: np.ndarray) -> dict:
    """img against the reference's two independent renders r1, r2 of the same
    spp (SURVEY.md §8(c) criterion 3): mean per-pixel RGB-L2 distance and the
    reference's own seed-to-seed floor, image-mean bias against 3 sigma of the
    mean estimator, and the 8x8-box-downsampled relative L2 against each
    reference render and its seed-to-seed value."""
    img, r1, r2 = (x.astype(np.float64) for x in (img, r1, r2))
    n = r1.shape[0] * r1.shape[1]
    return {
        "l2": float(np.linalg.norm(img - r1, axis=2).mean()),
        "l2_floor": float(np.linalg.norm(r1 - r2, axis=2).mean()),
        "bias": float(abs(img.mean() - r1.mean())),
        "sigma": float((r1 - r2).mean(axis=2).std() / np.sqrt(n)),
        "down_rel": [downsampled_rel_l2(img, r1), downsampled_rel_l2(img, r2)],
        "down_rel_floor": downsampled_rel_l2(r1, r2),
    }


# SURVEY.md §8(c) criterion 3 at >= 256 spp: 8x8-box-downsampled relative L2 <= 2%
DOWN_REL_MAX = 0.02


def assert_statistical(rep: dict, high_spp: bool = False) -> None:
    assert rep["l2"] <= 1.10 * rep["l2_floor"], rep
    assert rep["bias"] <= 3 * rep["sigma"], rep
    if high_spp:
        assert max(rep["down_rel"]) <= DOWN_REL_MAX, rep
        # and no further from the reference than its own other seed, within 10%
        assert np.mean(rep["down_rel"]) <= 1.10 * rep["down_rel_floor"], rep


def have_ref() -> bool:
    return os.path.exists(REF_DRIVER) and os.path.isdir("/root/reference")
