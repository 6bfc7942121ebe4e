#!/usr/bin/env python3
"""Diagnostic: WHY a sampled tile's pixels miss the near-exact bar.

For one 32x32 tile of a BASELINE workload, renders the tile on the GPU and in
the restatement (counter RNG, the same draws in the same order), takes the
pixels that are not within 1e-3 relative, and for each of them compares the
two renderers SAMPLE BY SAMPLE: the restatement's per-sample radiance
(rs_pixel_samples) against the GPU's (one launch per sample index: spp = 1,
pt_params.sample_base = i).  A pixel whose difference comes from a single
sample whose path took another turn (a silhouette hit decided differently in
fp32 than in fp64, or an occlusion test at grazing incidence) shows exactly
one differing sample, and that sample's difference / spp equals the pixel's.
Usage: python tools/silhouette_samples.py [--workload c4] [--tile 1088,192] [--seed 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--tile", default="1088,192")
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    from dsgpuraytracing_amd import scene_loader
    from dsgpuraytracing_amd.pathtracer import Device, Scene
    from tests.oracle_helpers import Restatement
    from tests.test_gpu_fullsize import THREADS, _workload, near_exact

    dae, env, w, h, spp = _workload(args.workload)
    tx, ty = map(int, args.tile.split(","))
    tw, th = min(32, w - tx), min(32, h - ty)
    rs = Restatement()
    with tempfile.TemporaryDirectory() as td:
        dump = scene_loader.dump_dae(dae, w, h, os.path.join(td, "scene.ptd"), envmap=env)
        ti = (ty // 32) * ((w + 31) // 32) + tx // 32
        ref, _ = rs.render(dump, w, h, spp, 4, 1, args.seed, rng_mode=1, threads=THREADS, tile_begin=ti,
                           tile_end=ti + 1)
        ref = ref[ty:ty + th, tx:tx + tw]
        dev = Device(0)
        dev.upload_scene(Scene.from_dump(dump))
        dev.set_camera(Scene.from_dump(dump).camera)
        dev.set_params(w, h, spp, 4, 1, args.seed)
        img = np.zeros((h, w, 3), np.float32)
        dev.render_tiles([(tx, ty, tw, th)], img)
        got = img[ty:ty + th, tx:tx + tw]
        diff = np.abs(got - ref).max(axis=2)
        off = diff > 1e-3 * np.maximum(1.0, np.abs(ref).max(axis=2))
        ys, xs = np.nonzero(off)
        print(json.dumps({"workload": args.workload, "tile": [tx, ty], "spp": spp,
                          "near_exact": round(near_exact(got, ref), 5), "off_pixels": int(off.sum())}))
        if not off.any():
            return
        ref_s = rs.pixel_samples(dump, w, h, spp, xs + tx, ys + ty, seed=args.seed)
        gpu_s = np.zeros_like(ref_s)
        one = np.zeros((h, w, 3), np.float32)
        for i in range(spp):  # the GPU's sample i of every pixel of the tile
            dev.set_params(w, h, 1, 4, 1, args.seed, sample_base=i)
            dev.render_tiles([(tx, ty, tw, th)], one)
            gpu_s[:, i] = one[ys + ty, xs + tx]
        rows = []
        for k in range(len(xs)):
            d = np.abs(gpu_s[k] - ref_s[k]).max(axis=1)
            bad = np.nonzero(d > 1e-4 * np.maximum(1.0, np.abs(ref_s[k]).max(axis=1)))[0]
            explained = (gpu_s[k, bad] - ref_s[k, bad]).sum(axis=0) / spp
            rows.append({"pixel": [int(xs[k] + tx), int(ys[k] + ty)],
                         "pixel_diff": [round(float(v), 6) for v in (got[ys[k], xs[k]] - ref[ys[k], xs[k]])],
                         "differing_samples": bad.tolist(),
                         "their_diff_over_spp": [round(float(v), 6) for v in explained],
                         "gpu": [[round(float(v), 5) for v in gpu_s[k, i]] for i in bad[:4]],
                         "oracle": [[round(float(v), 5) for v in ref_s[k, i]] for i in bad[:4]]})
        for r in rows:
            print(json.dumps(r))
        n = np.array([len(r["differing_samples"]) for r in rows])
        print(json.dumps({"off_pixels": len(rows), "differing_samples_per_off_pixel": np.bincount(n).tolist(),
                          "max": int(n.max())}))


if __name__ == "__main__":
    main()
