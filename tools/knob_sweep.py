#!/usr/bin/env python3
"""Diagnostic: render-kernel time under the launch tuning knobs (environment
variables read per launch by pt_api.cpp: PT_WAVES_PER_CU, PT_SHADE_BATCH,
PT_SAMPLE_GROUP, PT_LEAF_WEIGHT), for the whole frame and for one rank's
share of an N-GPU split.
Usage: python tools/knob_sweep.py --workload c3 --share 8 \
         --grid "PT_WAVES_PER_CU=12,16,20" --grid "PT_SAMPLE_GROUP=1,2" """
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--share", type=int, default=0, help="N: time rank 0's share of an N-GPU split (0: whole frame)")
    ap.add_argument("--deal", default="mod")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--grid", action="append", default=[])
    args = ap.parse_args()
    import torch

    import bench
    from dsgpuraytracing_amd import scenes
    from dsgpuraytracing_amd.dist import TileExchange
    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    wl = bench.WORKLOADS[args.workload]
    W, H, SPP = wl["w"], wl["h"], wl["spp"]
    envmap = None
    if wl["scene"] == "sub1":
        dae = scenes.proxy_path(1)
    elif wl["scene"] == "c5":
        dae, envmap = scenes.c5_path(2), scenes.c5_envmap_path()
    else:
        dae = scenes.C1_DAE
    sc = Scene.from_dae(dae, W, H, envmap=envmap)
    dev = Device(0)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(W, H, SPP, bench.DEPTH, bench.NSL, bench.SEED)
    d = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    tiles = tile_fifo(W, H)
    if args.share > 1:
        ex = TileExchange(tiles, W, H, 0, args.share, d, deal=args.deal)
        arr = np.asarray(ex.mine, np.int32)
        out_ptr, packed = ex.packed.data_ptr(), True
    else:
        frame = torch.zeros((H, W, 3), dtype=torch.float32, device=d)
        arr = np.asarray(tiles, np.int32)
        out_ptr, packed = frame.data_ptr(), False
    axes = []
    for g in args.grid:
        k, v = g.split("=", 1)
        axes.append([(k, x) for x in v.split(",")])
    for combo in itertools.product(*axes):
        for k, v in combo:
            os.environ[k] = v
        dev.render_tiles_device(arr, out_ptr, stream, packed=packed)
        ks = []
        for _ in range(args.steps):
            dev.render_tiles_device(arr, out_ptr, stream, packed=packed)
            ks.append(dev.stats()["last_ms"])
        print(json.dumps({"knobs": dict(combo), "share": args.share, "kernel_ms": round(float(np.median(ks)), 4),
                          "min_ms": round(min(ks), 4)}), flush=True)
        for k, _ in combo:
            del os.environ[k]


if __name__ == "__main__":
    main()
