#!/usr/bin/env python3
"""Diagnostic: render time of one workload's frame against spp.

The slope of t(spp) is the steady-state cost per sample; the intercept is the
per-launch fixed cost (launch, ramp-up, and the drain tail in which waves run
out of work one by one).  Prints one JSON line per spp and a least-squares fit.
Usage: python tools/spp_sweep.py [--workload c3] [--spp 8,16,32,64,128,256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--spp", default="8,16,32,64,128,256")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    from dsgpuraytracing_amd import scenes
    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo

    wl = bench.WORKLOADS[args.workload]
    w, h = wl["w"], wl["h"]
    envmap = None
    if wl["scene"] == "sub1":
        dae = scenes.proxy_path(1)
    elif wl["scene"] == "c5":
        dae, envmap = scenes.c5_path(2), scenes.c5_envmap_path()
    else:
        dae = scenes.C1_DAE
    scene = Scene.from_dae(dae, w, h, envmap=envmap)
    dev = Device(0)
    dev.upload_scene(scene)
    dev.set_camera(scene.camera)
    tiles = np.asarray(tile_fifo(w, h), dtype=np.int32).reshape(-1, 4)
    frame = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    xs, ys = [], []
    for spp in [int(s) for s in args.spp.split(",")]:
        dev.set_params(w, h, spp, bench.DEPTH, bench.NSL, bench.SEED)
        for _ in range(2):
            dev.render_tiles_device(tiles, frame.data_ptr(), stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ks = []
        for _ in range(args.reps):
            dev.render_tiles_device(tiles, frame.data_ptr(), stream)
            ks.append(dev.stats()["last_ms"])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.reps * 1e3
        xs.append(spp)
        ys.append(ms)
        print(json.dumps({"spp": spp, "ms": round(ms, 4), "kernel_ms": round(float(np.mean(ks)), 4),
                          "Gsamples_s": round(w * h * spp / ms / 1e6, 3)}), flush=True)
    a, b = np.polyfit(np.asarray(xs, float), np.asarray(ys, float), 1)
    print(json.dumps({"fit_ms_per_spp": round(float(a), 5), "fit_fixed_ms": round(float(b), 4),
                      "steady_Gsamples_s": round(w * h / a / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
