#!/usr/bin/env python3
"""Diagnostic: launch shape of one stats render (pt_get_wave_trace).

Prints, in microseconds after the first wave started, the quantiles of wave
end times and of the time each wave first found the work queue empty, the
same per XCC, and the waves that ended last with their CU and sample counts.
Usage: python tools/wave_trace.py [--workload c3] [--out gpurun_out/wave_trace.npy]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def st_group(st):
    """samples per work slot of the launch (slot latencies are summed per slot,
    samples per camera ray)"""
    return st["group_spp"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--out", default=None)
    ap.add_argument("--share", type=int, default=0, help="N: rank 0's share of an N-GPU split (packed output)")
    ap.add_argument("--census", action="store_true",
                    help="the PLAIN build's residency and drain instead: wave starts / first empty queue / ends "
                         "per CU, lanes alive and rounds in the drain; needs a library built with "
                         "PT_HIPCC_FLAGS=-DPT_CENSUS=1 (tools/variants.sh)")
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
    dev.set_params(w, h, wl["spp"], bench.DEPTH, bench.NSL, bench.SEED)
    tiles = np.asarray(tile_fifo(w, h), dtype=np.int32).reshape(-1, 4)
    frame = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    out_ptr, packed = frame.data_ptr(), False
    if args.share > 1:
        from dsgpuraytracing_amd.dist import TileExchange
        ex = TileExchange(tile_fifo(w, h), w, h, 0, args.share, frame.device)
        tiles = np.asarray(ex.mine, np.int32)
        out_ptr, packed = ex.packed.data_ptr(), True
    if args.census:
        os.environ["PT_CENSUS"] = "1"
        for _ in range(3):  # lone launches: each synchronised before the next
            dev.render_tiles_device(tiles, out_ptr, stream, packed=packed)
            torch.cuda.synchronize()
        tr = dev.wave_trace()
        t0 = tr[:, 0].min()
        start = (tr[:, 0] - t0) * 0.01
        end = (tr[:, 2] - t0) * 0.01
        xcc = (tr[:, 3] >> 32) & 0xF
        hw = tr[:, 3] & 0xFFFFFFFF
        cu_key = xcc * 256 + ((hw >> 8) & 0xFF)  # XCC, then HW_ID's CU / SH / SE fields
        early = start < 100.0
        per_cu = np.bincount(np.unique(cu_key[early], return_inverse=True)[1])
        q = [0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0]
        if not tr[:, 1].any():
            sys.exit("the library has no drain census: build it with PT_HIPCC_FLAGS=-DPT_CENSUS=1")
        emp = np.where(tr[:, 1] != -1, (tr[:, 1] - t0) * 0.01, np.nan)  # (-1: never saw it empty)
        print(json.dumps({"census": True, "waves": len(tr), "kernel_ms": dev.launch_times(1)[0][0].item(),
                          "start_us_quantiles": [round(float(np.quantile(start, x)), 1) for x in q],
                          "end_us_quantiles": [round(float(np.quantile(end, x)), 1) for x in q],
                          "empty_us_quantiles": [round(float(np.nanquantile(emp, x)), 1) for x in q],
                          "drain_us_quantiles": [round(float(np.nanquantile(end - emp, x)), 1) for x in q],
                          "alive_at_empty_quantiles": [int(np.quantile(tr[:, 4], x)) for x in q],
                          "drain_rounds_quantiles": [int(np.quantile(tr[:, 5], x)) for x in q],
                          # queue claims (atomics on the head): wait per claim, per wave's total, the longest
                          "claims_per_wave_mean": round(float(tr[:, 7].mean()), 2),
                          "claim_wait_us_mean": round(float(tr[:, 6].sum() / max(1, tr[:, 7].sum()) * 0.01), 3),
                          "claim_wait_us_per_wave_quantiles": [round(float(np.quantile(tr[:, 6] * 0.01, x)), 1) for x in q],
                          "claim_wait_max_us_quantiles": [round(float(np.quantile(tr[:, 8] * 0.01, x)), 2) for x in q],
                          "alive_at_empty_hist8": np.bincount(np.clip(tr[:, 4], 0, 64) // 8, minlength=9).tolist(),
                          "late_starts": int((~early).sum()), "cus_seen": int(len(np.unique(cu_key))),
                          "early_waves_per_cu_min_max": [int(per_cu.min()), int(per_cu.max())],
                          "early_waves_per_cu_hist": np.bincount(per_cu).tolist()}))
        return
    for _ in range(2):
        dev.render_tiles_device(tiles, out_ptr, stream, stats=True, packed=packed)
    torch.cuda.synchronize()
    st = dev.stats()
    tr = dev.wave_trace()
    if args.out:
        np.save(args.out, tr)
    t0 = tr[:, 0].min()
    us = 0.01  # device wall clock: 100 MHz
    end = (tr[:, 2] - t0) * us
    emp = np.where(tr[:, 1] > 0, (tr[:, 1] - t0) * us, np.nan)
    xcc = (tr[:, 3] >> 32) & 0xF
    hw = tr[:, 3] & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    q = [0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0]
    start = (tr[:, 0] - t0) * us
    out = {"kernel_ms": st["last_ms"], "waves": len(tr), "group_spp": st["group_spp"],
           "start_us_quantiles": [round(float(np.quantile(start, x)), 1) for x in q],
           "late_starts": int((start > 100.0).sum()),
           "end_us_quantiles": [round(float(np.quantile(end, x)), 1) for x in q],
           "empty_us_quantiles": [round(float(np.nanquantile(emp, x)), 1) for x in q],
           "samples_per_wave_quantiles": [int(np.quantile(tr[:, 4], x)) for x in q],
           "slot_latency_us_mean": round(float(tr[:, 5].sum() / max(1, tr[:, 4].sum()) * st_group(st) * us), 1),
           "slot_latency_us_max_quantiles": [round(float(np.quantile(tr[:, 6], x)) * us, 1) for x in q],
           "ray_steps_max_quantiles": [int(np.quantile(tr[:, 7] >> 32, x)) for x in q],
           "ray_idle_max_quantiles": [int(np.quantile(tr[:, 7] & 0xFFFFFFFF, x)) for x in q],
           "ray_rounds_max_quantiles": [int(np.quantile(tr[:, 8], x)) for x in q],
           "rounds_per_wave": st["wave_rounds"] / len(tr), "round_us": round(float(np.mean(end)) / (st["wave_rounds"] / len(tr)), 2),
           "drain_iters_per_wave_quantiles": [int(np.quantile(tr[:, 9], x)) for x in q],
           "drain_rounds_per_wave_quantiles": [int(np.quantile(tr[:, 10], x)) for x in q],
           "slot_latency_hist_log2us": st["slot_latency_hist"]}
    print(json.dumps(out))
    for x in range(8):
        m = xcc == x
        if m.any():
            print(json.dumps({"xcc": x, "waves": int(m.sum()),
                              "end_us_p50_p100": [round(float(np.quantile(end[m], 0.5)), 1), round(float(end[m].max()), 1)],
                              "empty_us_p50_p100": [round(float(np.nanquantile(emp[m], 0.5)), 1),
                                                    round(float(np.nanmax(emp[m])), 1)],
                              "samples": int(tr[m, 4].sum())}))
    late = np.argsort(-end)[:10]
    for i in late:
        print(json.dumps({"wave": int(i), "end_us": round(float(end[i]), 1), "empty_us": round(float(emp[i]), 1),
                          "xcc": int(xcc[i]), "se": int(se[i]), "cu": int(cu[i]), "samples": int(tr[i, 4])}))
    # end-time histogram, 25 bins
    hist, edges = np.histogram(end, bins=25)
    print(json.dumps({"end_hist_edges_us": [round(float(e), 1) for e in edges], "end_hist": hist.tolist()}))


if __name__ == "__main__":
    main()
