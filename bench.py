#!/usr/bin/env python3
"""Benchmark of the path-tracing hot path on MI355X.

Metric (BASELINE.json): "Mrays/sec + wall-clock render time, CBdragon 1024x1024
@ 64 spp".  A "step" is one full-frame render (every 32x32 tile of the
reference's FIFO) of a BASELINE config with max_ray_depth 4, ns_area_light 1
(readme.txt:1 settings).  Mrays/s = W*H*spp*frames / seconds / 1e6 (primary
path samples, the unit of the reference's "Primary (M ray/s)" column); scene
load / BVH build / upload are outside the timed region, as in the reference's
timers.  Samples whose camera ray provably misses the scene box (screen
footprint cull, exact) count as rendered, as in the reference's own unit; the
line also reports ray casts/s and a framed variant in which every pixel sees
the scene.

  * N = 1 (default): C3 = CBdragon proxy CBbunny_sub1 (114,316 triangles;
    CBdragon.dae is absent), 1024x1024, 64 spp.
  * N > 1 (torchrun, one process per GPU), default: the SAME C3 frame split
    over the GPUs ("scaling": "strong", north_star's "near-linear tile
    scaling"): the frame's 32x32 tiles dealt diagonally, each rank rendering
    its tiles into a packed buffer, then ONE RCCL gather of the packed tiles
    onto rank 0, pipelined: frame k's gather + scatter are
    queued behind its resolve on the current stream while frame k+1 renders
    on the library's render-slot streams (dist.PipelinedExchange); value = W*H*64 *
    frames / max-rank time, the image bit-identical to the 1-GPU image.
    `efficiency` = value / (N * rate_1), rate_1 measured by rank 0 rendering
    the whole frame alone behind a barrier (null when ranks share a device).
    Companions: BASELINE C4 (1080p, 256 spp) split the same way, and the weak
    C3 pass (each rank one 64-spp pass over disjoint sample indices + one
    RCCL sum-reduce; `--scaling weak` makes it the value).
The exchange is inside the timed region.  Device renders are queued back to
back and consecutive frames overlap on the GPU (pt_api.cpp's two-slot render
pipeline: the next frame's waves fill the CUs the previous frame's drain
leaves idle); config.single_frame_ms is the wall-clock time of one frame
rendered alone, synchronised on both sides.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# BASELINE.json configs; C3 is the headline (N = 1 default),
# C4 the multi-GPU default.  c3f: C3 with a camera framing the box interior.
WORKLOADS = {
    "c1": dict(scene="c1", w=256, h=256, spp=1, desc="C1 CBspheres_lambertian 256x256 1spp -m 4 -l 1"),
    "c2": dict(scene="c1", w=512, h=512, spp=16, desc="C2 CBspheres_lambertian 512x512 16spp -m 4 -l 1"),
    "c3": dict(scene="sub1", w=1024, h=1024, spp=64,
               desc="C3 CBbunny_sub1 (114,316 tris; CBdragon proxy) 1024x1024 64spp -m 4 -l 1, default camera"),
    "c3f": dict(scene="sub1", w=1024, h=1024, spp=64, cam="cam_bunny_framed.info",
                desc="C3 CBbunny_sub1 1024x1024 64spp -m 4 -l 1, camera framing the box interior "
                     "(assets/cam_bunny_framed.info: no pixel misses the scene)"),
    "c4": dict(scene="sub1", w=1920, h=1080, spp=256,
               desc="C4 CBbunny_sub1 (CBdragon proxy) 1920x1080 256spp -m 4 -l 1, default camera, tiles over N GPUs"),
    "c5": dict(scene="c5", w=1920, h=1080, spp=512,
               desc="C5 CBbunny_sub2_c5 (457,228 tris, glass bunny + mirror sphere; CBlucy proxy) + synthetic "
                    "512x256 environment light, 1920x1080 512spp -m 4 -l 1, tiles over N GPUs"),
    # C5 at BASELINE.json's "~1M tris" scale (sub3 ~1.83M)
    "c5big": dict(scene="c5big", w=1920, h=1080, spp=512,
                  desc="C5 CBbunny_sub3_c5 (1,828,877 tris, glass bunny + mirror sphere; CBlucy proxy at BASELINE's "
                       "~1M-tri scale) + synthetic 512x256 environment light, 1920x1080 512spp -m 4 -l 1"),
}
HEADLINE_METRIC = "Mrays/sec + wall-clock render time, CBdragon 1024x1024 @ 64 spp"
W, H, SPP, DEPTH, NSL, SEED = 1024, 1024, 64, 4, 1, 1
# MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec; L2 34.5 TB/s aggregate (8 XCDs);
# VALU: each SIMD issues one wave64 VALU instruction per 2 cycles -> 2 per CU
# per cycle, 256 CUs at 2.4 GHz.
HBM_PEAK_GBS = 8000.0
L2_PEAK_GBS = 34500.0
VALU_PEAK_GINST = 256 * 2 * 2.4
L2_LINE = 128


def workload_scene(wl):
    from dsgpuraytracing_amd import scenes
    if wl["scene"] == "sub1":
        dae, envmap = scenes.proxy_path(1), None
    elif wl["scene"] == "c5":
        dae, envmap = scenes.c5_path(2), scenes.c5_envmap_path()
    elif wl["scene"] == "c5big":
        dae, envmap = scenes.c5_path(3), scenes.c5_envmap_path()
    else:
        dae, envmap = scenes.C1_DAE, None
    cam = os.path.join(ROOT, "assets", wl["cam"]) if wl.get("cam") else None
    return dae, envmap, cam


def algorithmic_bytes(st: dict) -> float:
    """SURVEY.md §8(d) reference-layout cost model: 64 B per BVH node visit,
    48 B per triangle test, 16 B per sphere test, 4 B per leaf primitive index,
    36 B per hit (vertex normals), 12 B per pixel written.  The counts are
    those of the reference's binary BVH (PT_FLAG_REF_COUNTS launch).  The scene
    is L2 / Infinity-Cache resident, so these bytes are CACHE-SERVED: they are
    priced against the L2 roof, never against HBM."""
    prim = st["tri_tests"] + st["sphere_tests"]
    return (64.0 * st["node_visits"] + 48.0 * st["tri_tests"] + 16.0 * st["sphere_tests"] + 4.0 * prim
            + 36.0 * st["ext_hits"] + 12.0 * st["pixels"])


def lib_path() -> str:
    from dsgpuraytracing_amd import native
    return os.path.abspath(os.environ["PT_LIB"]) if os.environ.get("PT_LIB") else native.LIB_PATH


def kernel_sha256(path=None) -> str:
    """sha256 of the device code (.hip_fatbin) of the libptgpu.so this process
    loads: what a PMC summary's counts belong to (dsgpuraytracing_amd/elfsha.py)."""
    from dsgpuraytracing_amd import elfsha
    return elfsha.kernel_sha256(path or lib_path())


def lib_sha256(path=None) -> str:
    """sha256 of the libptgpu.so this process loads (PT_LIB or the in-tree one)."""
    import hashlib
    path = path or lib_path()
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def profile_summary(workload: str):
    """PMC summary of the render kernel on this workload (tools/profile_summary.py
    -> profiles/<round>/<workload>_summary.json; the newest round wins)."""
    pdir = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r") and d[1:].isdigit()),
                    key=lambda d: int(d[1:]), reverse=True) if os.path.isdir(pdir) else []
    for r in rounds:
        p = os.path.join(pdir, r, f"{workload}_summary.json")
        if os.path.exists(p):
            with open(p) as f:
                d = json.load(f)
            d["source"] = os.path.relpath(p, ROOT)
            return d
    return None


def roofline(workload: str, frame_ms: float, alg_bytes: float, isolated_ms: float = 0.0,
             pipelined_ms: float = 0.0, lib_sha: str | None = None, kernel_sha: str | None = None) -> dict:
    """Roofline of the dominant kernel (render_kernel).  Per-launch counts come
    from the committed PMC summary of the same workload and library (they are a
    property of the workload and the build, not of the clock; `pmc_stale` is
    true when the summary was collected on a different libptgpu.so than the one
    this run loaded: the device-code sha256, `kernel_sha256`, when the summary
    carries one, else the whole library's).  Views:
      hbm   -- (2 x FETCH_SIZE + WRITE_SIZE) bytes (gfx950 correction,
               MI355X_MICROARCH.md §HBM) vs 8 TB/s;
      l2    -- (TCC_HIT + TCC_MISS) requests x 128 B vs 34.5 TB/s (an upper
               bound of the bytes the L2 served);
      valu  -- SQ_INSTS_VALU wave-instructions vs 2 per CU per cycle;
      algorithmic -- the §8(d) cost-model bytes, cache-served, vs the L2 roof.
    Rates: `frac` (and `achieved`) divide the counts of one frame's launch by
    the measured frame interval ms_per_step (`frame_ms`) -- consecutive frames
    overlap on the GPU (pt_api.cpp's two-slot render pipeline), so the frame
    interval, not an event span, is the time one launch's work occupies the
    chip; `frac_isolated` divides them by the kernel's duration when it runs
    alone (`isolated_ms`: HIP events around lone, synchronised frames; the
    PT_PIPELINE=0 rocprofv3 kernel trace in profiles/ agrees with it).
    `pipelined_launch_ms` is the HIP-event span of a launch in the timed
    region: it includes waiting for the other render slot's CUs and is not a
    kernel duration.  `bound` names the measured view with the highest
    fraction; the kernel is latency-bound below all of them (SQ_WAIT_ANY)."""
    t = frame_ms * 1e-3
    ti = isolated_ms * 1e-3 if isolated_ms > 0 else None
    pm = profile_summary(workload)
    views = {}

    def view(name, per_launch, peak, unit, key="bytes_per_launch", **extra):
        a = per_launch / t / 1e9
        v = {key: per_launch, "achieved": round(a, 1), "peak": peak, "unit": unit, "frac": round(a / peak, 4)}
        if ti:
            v["frac_isolated"] = round(per_launch / ti / 1e9 / peak, 4)
        v.update(extra)
        views[name] = v

    view("algorithmic_cache_served", alg_bytes, L2_PEAK_GBS, "GB/s")
    hbm_bytes = None
    if pm:
        if "hbm_bytes_per_launch" in pm:
            hbm_bytes = pm["hbm_bytes_per_launch"]
            view("hbm", hbm_bytes, HBM_PEAK_GBS, "GB/s")
        tcc = pm.get("tcc", {})
        if "TCC_HIT_sum" in tcc and "TCC_MISS_sum" in tcc:
            view("l2", (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]) * L2_LINE, L2_PEAK_GBS, "GB/s",
                 hit_rate=round(pm.get("l2_hit_rate", 0.0), 4))
        sq = pm.get("sq", {})
        if "SQ_INSTS_VALU" in sq:
            view("valu", sq["SQ_INSTS_VALU"], VALU_PEAK_GINST, "G wave-instructions/s", key="insts_per_launch")
    measured = [k for k in ("hbm", "l2", "valu") if k in views]
    bound = max(measured, key=lambda k: views[k]["frac"]) if measured else "algorithmic_cache_served"
    v = views[bound]
    out = {"bound": bound, "achieved": v["achieved"], "peak": v["peak"], "unit": v["unit"], "frac": v["frac"],
           "frac_isolated": v.get("frac_isolated"), "traffic": hbm_bytes, "duration_ms": round(frame_ms, 4),
           "isolated_kernel_ms": round(isolated_ms, 4) if isolated_ms else None,
           "pipelined_launch_ms": round(pipelined_ms, 4) if pipelined_ms else None, "views": views}
    if pm:
        out["pmc"] = {k: (round(pm[k], 4) if isinstance(pm.get(k), float) else pm.get(k))
                      for k in ("avg_ms", "isolated_avg_ms", "sq_wait_any_frac", "sq_wait_inst_any_frac",
                                "sq_active_inst_any_frac", "valu_issue_util", "l2_hit_rate", "source", "lib_sha256",
                                "kernel_sha256")}
        # stale = the counts were collected on different device code than this
        # run's (summaries without a kernel stamp compare the whole library)
        if pm.get("kernel_sha256") and kernel_sha:
            out["pmc_stale"] = pm["kernel_sha256"] != kernel_sha
        else:
            out["pmc_stale"] = bool(lib_sha) and pm.get("lib_sha256") != lib_sha
    return out


REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")


def _coprime(k, ntx):
    import math
    while k > 1 and math.gcd(k, ntx) != 1:  # strides sharing a factor with the row length sample columns
        k += 1
    return k


def cpu_baseline_reference(dae: str, envmap, budget_s: float = 15.0, threads: int = 1) -> dict:
    """The reference's OWN CPU path (oracle/_ref/ref_driver, compiled from
    /root/reference/src by oracle/ref/Makefile; it travels to the GPU box with
    the tree) timed on this host: PathTracer::raytrace_tile (pathtracer.cpp:
    585-611) on every k-th 32x32 tile of the frame's FIFO, k sized from a
    calibration run so the sample takes about budget_s.  threads = 1: one
    thread with glibc rand() as shipped (== its -t 1 setting); threads = T:
    T threads popping the sample's tiles from one shared queue as its
    worker_thread does (pathtracer.cpp:613-637) -- readme.txt:1 publishes
    -t 8, where the shared rand() lock keeps it near the -t 1 rate.  Scene
    load and BVH build are excluded, as in the reference's own timer."""
    import subprocess

    ntx = (W + 31) // 32
    ntiles = ntx * ((H + 31) // 32)

    def run(begin, stride):
        cmd = [REF_DRIVER, dae, "--mode", "tiles", "-w", str(W), "-h", str(H), "-s", str(SPP), "-m", str(DEPTH),
               "-l", str(NSL), "--seed", str(SEED), "--tile-begin", str(begin), "--tile-stride", str(stride),
               "-t", str(threads)]
        if envmap:
            cmd += ["--envmap", envmap]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=600, check=True)
        return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])

    cal = _coprime(max(1, ntiles // 12), ntx)
    c = run(cal // 2, cal)
    per_tile = max(c["render_s"], 1e-4) / max(1, c["tiles"])
    step = _coprime(max(1, int(round(ntiles * per_tile / budget_s))), ntx)
    m = run(step // 2, step)
    how = ("one thread, glibc rand() as shipped (its -t 1)" if threads == 1 else
           f"{threads} threads on one shared tile queue as its worker_thread, glibc rand() as shipped (its -t {threads}, "
           f"readme.txt:1's published setting)")
    return {"value": m["pixels"] * SPP / m["render_s"] / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "reference",
            "sample": f"every {step}th 32x32 tile of the {W}x{H} frame ({m['pixels']} px, uniform) at {SPP} spp, "
                      f"-m {DEPTH} -l {NSL}: the reference's PathTracer::raytrace_tile built from its own sources "
                      f"(oracle/_ref/ref_driver --mode tiles), {how}, {m['render_s']:.1f} s of rendering"}


def _tiles_px(begin, stride):
    ntx = (W + 31) // 32
    ntiles = ntx * ((H + 31) // 32)
    px = 0
    for ti in range(begin, ntiles, stride):
        tx, ty = (ti % ntx) * 32, (ti // ntx) * 32
        px += (min(W, tx + 32) - tx) * (min(H, ty + 32) - ty)
    return px


def cpu_baseline_port(scene_dump: str, budget_s: float = 12.0, rng_mode: int = 0, threads: int = 1) -> dict:
    """The reference CPU algorithm as restated in oracle/restate.cpp, timed on
    this host on a bounded, UNIFORM sample of the same workload: every k-th
    tile of the 32x32 tile FIFO at the full spp, k sized from a calibration
    run so the sample takes about budget_s (scene load excluded).
      rng_mode 0, 1 thread: glibc rand(), bit-identical to the reference at -t 1;
      rng_mode 1, T threads: the counter RNG (no shared rand() lock), the
        "fair" CPU baseline of BASELINE.md §3 -- the same algorithm scaled
        over the host cores the GPU job owns."""
    from tests.oracle_helpers import Restatement
    rs = Restatement()
    ntx = (W + 31) // 32
    ntiles = ntx * ((H + 31) // 32)
    cal = _coprime(max(1, ntiles // 16), ntx)
    _, _, t_cal = rs.render_strided(scene_dump, W, H, SPP, DEPTH, NSL, SEED, rng_mode=rng_mode, threads=threads,
                                    tile_begin=cal // 2, tile_stride=cal)
    per_tile = max(t_cal, 1e-4) / len(range(cal // 2, ntiles, cal))
    step = _coprime(max(1, int(round(ntiles * per_tile / budget_s))), ntx)
    _, _, secs = rs.render_strided(scene_dump, W, H, SPP, DEPTH, NSL, SEED, rng_mode=rng_mode, threads=threads,
                                   tile_begin=step // 2, tile_stride=step)
    px = _tiles_px(step // 2, step)
    rng = "glibc-rand mode (== reference -t 1)" if rng_mode == 0 else "counter-RNG mode"
    return {"value": px * SPP / secs / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"every {step}th 32x32 tile of the {W}x{H} frame ({px} px, uniform) at {SPP} spp, -m {DEPTH} "
                      f"-l {NSL}, oracle/restate.cpp {rng}, {threads} thread(s), {secs:.1f} s of rendering"}


def host_threads() -> int:
    """Host threads this job may use: the affinity set, capped at 16 (the GPU
    box's CPU share per GPU; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scene-dump", default=None, help="PTDUMP scene instead of the native .dae loader")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the companion measurements (N = 1: framed C3, single-GPU C4 and C5, host-SAH tree, "
                         "per-tile seams; N > 1: the C4 frame split and the weak C3 pass)")
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: c3 (the headline config) at every N")
    ap.add_argument("--lbvh", action="store_true", help="build the BVH on the GPU (pt_upload_scene_lbvh)")
    ap.add_argument("--spp", type=int, default=0, help="diagnostic: override the workload's spp (not a BASELINE config)")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="diagnostic: render only one rank's share of an N-GPU split on this one GPU")
    ap.add_argument("--emulate-rank", type=int, default=0, help="the rank --emulate-shard renders")
    ap.add_argument("--split-tile", type=int, default=32,
                    help="tile edge of the strong split's deal (16 or 32; the reference's FIFO is 32x32): "
                         "smaller tiles spread each rank's share more evenly over the frame")
    ap.add_argument("--tile", type=int, default=32,
                    help="diagnostic: tile edge of the one-GPU (and weak) tile FIFO (8, 16 or 32)")
    ap.add_argument("--tile-order", default="rows", choices=["rows", "morton"],
                    help="diagnostic: order of the tile FIFO (rows: the reference's row-major queue; morton: "
                         "Z-order of the tiles) -- the same image in any order")
    ap.add_argument("--deal-block", type=int, default=0,
                    help="edge of the blocks the strong split deals (default: --split-tile); 16x16 tiles dealt "
                         "by 32x32 blocks keep each block's four tiles on one rank")
    ap.add_argument("--split-deal", default="auto",
                    help="the strong split's tile deal (dist.tile_owner: auto = diag3 at N >= 8, diag below; diag, "
                         "diagK, mod)")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames rendered per launch (pt_render_frames_device, 1..8; the library renders frames "
                         "of more than 32 work slots per lane one per launch): a frame batch shares one "
                         "persistent launch, so a small frame's drain is filled with the next frame's work. "
                         "Default 8 (the weak pass: 1)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="N > 1: strong = one frame's tiles split across the GPUs + one pipelined RCCL gather "
                         "(default; BASELINE C4: --workload c4); weak = one pass of the whole frame per GPU over "
                         "disjoint sample ranges + one RCCL reduce")
    args = ap.parse_args()
    if os.environ.get("PT_BENCH_LBVH") == "1":  # A/B arms (tools/ab.sh): the GPU-built tree
        args.lbvh = True

    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.dist import (PipelinedExchange, RankFailure, StepGuard, check_value_knobs, init_from_env,
                                          shard_tiles)
    # PT_DIST_BACKEND=gloo + PT_BENCH_DEVICE=0: rehearsal of the N-rank flow
    # with every rank on one GPU (the exchange then stages through host memory)
    backend = os.environ.get("PT_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PT_BENCH_DEVICE") is not None:
        local = int(os.environ["PT_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    # A dedicated current stream: renders are queued on it (pt_render_tiles_device
    # would put a NULL stream on the context's own non-blocking stream), so torch
    # ops and the RCCL collectives, which follow the current stream, see the
    # finished frame.
    torch.cuda.set_stream(torch.cuda.Stream(device=local))
    rank, world, _ = init_from_env(backend)
    try:
        bench_run(args, backend, local, rank, world, StepGuard, PipelinedExchange, check_value_knobs, shard_tiles)
    except RankFailure as e:
        # every rank raises it (dist.agree_status): report, leave the group, exit non-zero
        print(f"[bench rank {rank}] aborted: {e}", file=sys.stderr, flush=True)
        if rank == 0:
            print(json.dumps({"metric": HEADLINE_METRIC, "value": None, "error": str(e), "n_gpus": world}), flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()
        sys.exit(3)
    if dist.is_initialized():
        dist.destroy_process_group()


def ordered_tiles(tiles, order="rows"):
    """The tile FIFO in `order`: "rows" keeps the reference's row-major queue
    (pathtracer.cpp:209-214); "morton" sorts the tiles by the Z-order of their
    (column, row) -- a launch's blocks follow its tile list, so the order sets
    which pixels the waves in flight share.  Images are per pixel and sample:
    identical in any order."""
    if order == "rows" or not tiles:
        return list(tiles)
    t = max(max(w, h) for (_, _, w, h) in tiles)  # (the tile edge; clipped edge tiles are smaller)

    def z(tile):
        c, r, k = tile[0] // t, tile[1] // t, 0
        for b in range(16):
            k |= ((c >> b) & 1) << (2 * b) | ((r >> b) & 1) << (2 * b + 1)
        return k
    return sorted(tiles, key=z)


def xchg_opts():
    """The strong split's exchange: on the current stream behind the resolve
    (default), or on a side stream with PT_XCHG_SIDE=1 (A/Bs:
    profiles/r6/ab_stream_queues.txt)."""
    return {"side": os.environ.get("PT_XCHG_SIDE", "0") == "1"}


def bench_run(args, backend, local, rank, world, StepGuard, PipelinedExchange, check_value_knobs, shard_tiles):
    import torch
    import torch.distributed as dist

    global W, H, SPP
    workload = args.workload or "c3"
    wl = WORKLOADS[workload]
    W, H, SPP = wl["w"], wl["h"], args.spp or wl["spp"]

    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo

    t_load = time.perf_counter()
    dae, envmap, cam = None, None, None
    if args.scene_dump:
        scene = Scene.from_dump(args.scene_dump)
        dump_path = args.scene_dump
    else:
        dae, envmap, cam = workload_scene(wl)
        scene = Scene.from_dae(dae, W, H, cam_info=cam, envmap=envmap)
        dump_path = None
    dev = Device(local)
    t_up = time.perf_counter()
    dev.upload_scene(scene, gpu_bvh=args.lbvh)
    t_up = time.perf_counter() - t_up
    dev.set_camera(scene.camera)
    weak = world > 1 and args.scaling == "weak"
    # weak: this rank's pass covers sample indices SPP*rank .. SPP*rank+SPP-1
    dev.set_params(W, H, SPP, DEPTH, NSL, SEED, sample_base=SPP * rank if weak else 0)
    t_load = time.perf_counter() - t_load

    # the strong split deals tiles of --split-tile pixels (the same image for
    # any tiling: values are per pixel and sample)
    split = world > 1 and not weak or args.emulate_shard > 1
    tiles = ordered_tiles(tile_fifo(W, H, args.split_tile if split else args.tile), args.tile_order)
    frame = torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream().cuda_stream

    # strong: this rank's share of the tiles; weak (and one GPU): every tile
    mine_arr = np.asarray(tiles, dtype=np.int32).reshape(-1, 4)
    if args.emulate_shard > 1:
        mine_arr = np.asarray(shard_tiles(tiles, args.emulate_rank, args.emulate_shard, args.split_deal,
                                          args.deal_block or args.split_tile),
                              dtype=np.int32).reshape(-1, 4)
    # strong: packed tiles, the gather queued behind each frame's resolve
    fpl = 1 if weak else max(1, min(8, args.frames_per_launch or 8))
    pex = (PipelinedExchange(tiles, W, H, rank, world, frame.device, buffers=max(2, fpl), deal=args.split_deal,
                             tile_size=args.split_tile, deal_block=args.deal_block, **xchg_opts())
           if world > 1 and not weak else None)
    if args.emulate_shard > 1:
        # one rank's share through the same packed render + exchange (here a
        # device copy of the share's packed tiles and their scatter -- through
        # a one-rank RCCL group with PT_DIST_FORCE=1 -- the gather's link time
        # is not in it), host overheads included
        pex = PipelinedExchange([tuple(int(v) for v in t) for t in mine_arr], W, H, 0, 1, frame.device,
                                buffers=max(2, fpl), tile_size=args.split_tile, **xchg_opts())
    if pex is not None:
        mine_arr = np.asarray(pex.mine, dtype=np.int32).reshape(-1, 4)

    band = [frame]  # weak: the rows the reduce carries (set from the launch's screen footprint below)

    def reduce_passes():  # weak: sum the N passes onto rank 0, mean over SPP*N samples
        rows = band[0]
        if rows.numel() == 0:
            return
        if backend == "gloo":  # host staging (one-GPU rehearsals)
            h = rows.cpu()
            dist.reduce(h, dst=0)
            if rank == 0:
                rows.copy_(h)
        else:
            dist.reduce(rows, dst=0)
        if rank == 0:
            rows.mul_(1.0 / world)

    xev = []  # (start, end) events around each timed step's exchange
    # A rank whose render fails keeps joining the exchanges; guard.check() (a
    # collective at the synchronisation points) then stops every rank with the
    # failing rank's error (dsgpuraytracing_amd.dist.RankFailure).
    guard = StepGuard()
    kframe = [0]  # frames issued (the strong split's packed buffer is frame % 2)

    def step(stats=False, timed=False):
        if pex is None:  # the whole tile FIFO straight into the frame (one GPU, or this rank's pass)
            guard.run(dev.render_tiles_device, mine_arr, frame.data_ptr(), stream, stats=stats)
            if weak:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
                reduce_passes()
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                if timed:
                    xev.append((e0, e1))
        else:  # this rank's tiles into a packed buffer, then one gather onto rank 0 off the render's stream
            k = kframe[0]
            kframe[0] += 1
            buf = pex.packed_for(k)
            guard.run(dev.render_tiles_device, mine_arr, buf.data_ptr(), stream, stats=stats, packed=pex.ex.slot,
                      out_floats=buf.numel())
            pex.exchange(k, frame, timed=timed)
        return guard.run(dev.stats) if stats else None

    def steps(n, timed=False):
        """n frames: with --frames-per-launch F > 1 in frame batches of up to F
        frames per launch (pt_render_frames_device; the same images), each
        frame then exchanged as step() does."""
        if fpl <= 1 or weak:
            for _ in range(n):
                step(timed=timed)
            return
        done = 0
        while done < n:
            m = min(fpl, n - done)
            if pex is None:
                guard.run(dev.render_frames_device, mine_arr, [frame.data_ptr()] * m, [SEED] * m, stream)
            else:
                ks = list(range(kframe[0], kframe[0] + m))
                kframe[0] += m
                bufs = [pex.packed_for(k) for k in ks]
                guard.run(dev.render_frames_device, mine_arr, [b.data_ptr() for b in bufs], [SEED] * m, stream,
                          packed=pex.ex.slot, out_floats=bufs[0].numel())
                for k in ks:
                    pex.exchange(k, frame, timed=timed)
            done += m

    # counters for the roofline's algorithmic bytes: the reference's binary BVH
    # (SURVEY.md §8(d) cost model); and the launch's own counters (4-wide BVH)
    st_counts = step(stats="ref")
    st_perf = step(stats=True)
    guard.check()
    if weak:
        # Rows outside the scene's screen footprint are 0 in every pass (their
        # camera rays miss the scene box: pt_stats.footprint), so the reduce
        # carries only the footprint's rows -- the same image, fewer bytes
        # (C3: 53% of the frame's rows).  Every rank computes the same rows.
        y0, y1 = st_perf["footprint"][1], st_perf["footprint"][3]
        if y1 < y0:  # the empty footprint (the box is off-screen): every pixel is 0, nothing to reduce
            y0, y1 = 0, -1
        band[0] = frame[y0:y1 + 1]
        frame[:y0].zero_()
        frame[y1 + 1:].zero_()
    # the ranks must group each pixel's samples alike (bit-identical frame)
    knobs = check_value_knobs({"group_spp": st_perf["group_spp"]})
    steps(args.warmup)
    guard.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps, timed=True)  # asynchronous: nothing waits on the GPU inside a step
    if pex is not None:
        pex.drain()  # (with PT_XCHG_SIDE=1: the current stream waits for the last side-stream exchange)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    guard.check()
    # HIP events recorded around every launch on its stream (the timed ones)
    n_launch = args.steps if fpl <= 1 or weak else -(-args.steps // fpl)
    kernel_ms, resolve_ms = dev.launch_times(n_launch)
    if n_launch != args.steps:  # (a frame batch's launch and resolves: per frame)
        kernel_ms, resolve_ms = kernel_ms * n_launch / args.steps, resolve_ms * n_launch / args.steps
    xchg_ms = float(np.mean([a.elapsed_time(b) for a, b in xev])) if xev else 0.0
    if pex is not None:
        xchg_ms = pex.exchange_ms()
    # strong split: the 1-GPU point of the curve, rank 0 rendering the whole
    # frame alone behind a barrier (the other ranks idle), same clock and frames
    rate1, shared = None, False
    if world > 1 and not weak:
        rate1, shared = single_gpu_rate(dev, tiles, W, H, SPP, frame, stream, rank, backend, args.steps, fpl=fpl)
    per_rank = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mine = torch.tensor([float(np.mean(kernel_ms)), float(np.mean(resolve_ms)), xchg_ms,
                             float(np.sum(mine_arr[:, 2] * mine_arr[:, 3])), float(st_perf["partial_bytes"]),
                             float(st_counts["culled_samples"])],
                            dtype=torch.float64, device="cpu" if backend == "gloo" else f"cuda:{local}")
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[round(float(v), 4) for v in r.cpu().tolist()] for r in allr]

    multi = None
    if world > 1 and not args.no_extras:
        # every rank takes part (collectives inside)
        multi = multi_gpu_companions(local, rank, world, backend, StepGuard, PipelinedExchange,
                                     frames=max(3, min(args.steps, 10)), with_weak=not weak,
                                     split_tile=args.split_tile, split_deal=args.split_deal,
                                     deal_block=args.deal_block)

    host_ms = None
    single_ms = None
    frame_batch = None
    iso_ms = 0.0
    iso_single_ms = None
    if world == 1:
        # one frame alone, synchronised on both sides (no overlap with a
        # neighbouring frame): the wall-clock render time of ONE frame, and
        # the render kernel's own duration (HIP events around a launch that
        # shares the GPU with nothing)
        lat, api, idle = [], [], []
        for _ in range(5):
            torch.cuda.synchronize()
            t0s = time.perf_counter()
            step()
            t1s = time.perf_counter()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0s)
            api.append(t1s - t0s)
            t2s = time.perf_counter()
            torch.cuda.synchronize()  # (an idle synchronize: the clock's own floor)
            idle.append(time.perf_counter() - t2s)
        single_ms = float(np.median(lat)) * 1e3
        single_api_ms = float(np.median(api)) * 1e3
        sync_floor_ms = float(np.median(idle)) * 1e3
        iso_ms = float(np.median(dev.launch_times(5)[0]))
        iso_single_ms = iso_ms
        if fpl > 1 and args.emulate_shard <= 1:
            # the timed kernel is the frame batch's: its own duration alone on
            # the GPU (a lone launch of fpl frames, synchronised on both sides),
            # per frame -- the roofline's isolated fraction divides the per-frame
            # counts of the same 8-frame launches (profiles/<round>/c3_summary.json)
            isb = []
            for _ in range(3):
                torch.cuda.synchronize()
                dev.render_frames_device(mine_arr, [frame.data_ptr()] * fpl, [SEED] * fpl, stream)
                torch.cuda.synchronize()
                nfl = dev.stats()["frames_per_launch"]
                if nfl <= 1:  # larger frames render one per launch: the lone single frame above
                    break
                isb.append(dev.launch_times(1)[0][0] / nfl)
            if isb:
                iso_ms = float(np.median(isb))
        # the drop-in pt_render_tiles path: output copied to a host buffer (PCIe-inclusive)
        host = np.zeros((H, W, 3), np.float32)
        dev.render_tiles(mine_arr, host)
        t0h = time.perf_counter()
        for _ in range(2):
            dev.render_tiles(mine_arr, host)
        host_ms = (time.perf_counter() - t0h) / 2 * 1e3
        # beside a batched line: the same frames one per launch
        # (pt_render_tiles_device per frame, the reference's one-frame call)
        if args.emulate_shard <= 1 and fpl > 1 and workload == "c3":  # (larger frames render one per launch anyway)
            nb = 32
            for _ in range(2):
                dev.render_tiles_device(mine_arr, frame.data_ptr(), stream)
            torch.cuda.synchronize()
            t0b = time.perf_counter()
            for _ in range(nb):
                dev.render_tiles_device(mine_arr, frame.data_ptr(), stream)
            torch.cuda.synchronize()
            elb = time.perf_counter() - t0b
            frame_batch = {"frames_per_launch": 1, "frames": nb, "ms_per_step": round(elb / nb * 1e3, 4),
                           "value": round(W * H * SPP * nb / elb / 1e6, 1)}
    if rank == 0:
        frames = args.steps
        value = W * H * SPP * frames * (world if weak else 1) / elapsed / 1e6
        if args.emulate_shard > 1:
            value = float(np.sum(mine_arr[:, 2] * mine_arr[:, 3])) * SPP * frames / elapsed / 1e6
        avg_ms = float(np.mean(kernel_ms))
        img = frame.float().cpu().numpy()
        # at N = 1 the line names the curve it starts (the driver's N > 1 runs
        # use the same default, the C3 frame split)
        scaling = "weak" if weak else "strong" if world > 1 else args.scaling
        out = {
            "metric": HEADLINE_METRIC if workload == "c3" else f"Mrays/sec + wall-clock render time, {wl['desc']}",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / frames * 1e3, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": {"c5": "synthetic: deterministic CBbunny_sub2 glass/mirror proxy for the missing CBlucy.dae + "
                           "seeded 512x256 environment map (SURVEY §8(d))",
                     "c5big": "synthetic: deterministic CBbunny_sub3 glass/mirror proxy (BASELINE's ~1M tris) for the "
                              "missing CBlucy.dae + seeded 512x256 environment map (SURVEY §8(d))",
                     "c1": "CBspheres_lambertian.dae from the reference", "c2": "CBspheres_lambertian.dae from the reference"
                     }.get(workload,
                           "synthetic: deterministic CBbunny_sub1 proxy for the missing CBdragon.dae (SURVEY §8(d))"),
            "config": {"workload": wl["desc"],
                       "width": W, "height": H, "spp": SPP, "max_ray_depth": DEPTH, "ns_area_light": NSL,
                       "spp_total": SPP * world if weak else SPP,
                       "parallelism": (f"samples{world}" if weak else f"tiles{world}") if world > 1 else "single",
                       "frames_per_launch": 1 if weak else fpl,
                       "exchange_bytes_per_rank": (int(band[0].numel() * 4) if weak else
                                                   (int(pex.ex.packed.numel() * 4) if pex is not None else 0)),
                       # BASELINE's "wall-clock render time": ONE frame start to image,
                       # synchronised on both sides (the reference's timer spans one
                       # render, application.cpp:776-780); the pipelined frame
                       # interval is ms_per_step
                       "render_time_s": round((single_ms if single_ms is not None else elapsed / frames * 1e3) / 1e3, 7),
                       "wall_clock_frame_ms": None if single_ms is None else round(single_ms, 3),
                       "pipelined_frame_interval_ms": round(elapsed / frames * 1e3, 4),
                       "scene_load_s": round(t_load, 3),
                       "single_frame_ms": None if single_ms is None else round(single_ms, 3),
                       # host time inside the render call (launch preparation) and an idle synchronize
                       "single_frame_api_ms": None if single_ms is None else round(single_api_ms, 4),
                       # the render kernel of ONE frame alone (one frame per launch, HIP events);
                       # roofline.isolated_kernel_ms is the timed launch's own: per frame of a lone batch
                       "single_frame_kernel_ms": None if iso_single_ms is None else round(iso_single_ms, 4),
                       "sync_floor_ms": None if single_ms is None else round(sync_floor_ms, 4),
                       "bvh": bvh_desc(args.lbvh),
                       "upload_s": round(t_up, 4),
                       "host_output_ms_per_frame": None if host_ms is None else round(host_ms, 3)},
            "roofline": roofline(workload, elapsed / frames * 1e3, algorithmic_bytes(st_counts), isolated_ms=iso_ms,
                                 pipelined_ms=avg_ms, lib_sha=lib_sha256(), kernel_sha=kernel_sha256()),
            "resolve_ms": round(float(np.mean(resolve_ms)), 4),
            "counters": {k: st_counts[k] for k in ("camera_rays", "bounce_rays", "shadow_rays", "node_visits",
                                                   "tri_tests", "sphere_tests", "ext_hits", "culled_samples")},
            "launch_counters": {k: st_perf[k] for k in ("node_visits", "tri_tests", "sphere_tests", "wave_trav_steps",
                                                        "leaf_steps", "wave_rounds", "queue_atomics", "shade_clocks",
                                                        "hitshade_clocks", "trav_clocks", "max_wave_clocks",
                                                        "wave_wall_sum", "wave_wall_max", "section_clocks", "wave_span",
                                                        "lane_iters", "partial_bytes", "deep_stack_steps",
                                                        "node_census")},
            # frames per timed launch: the roofline's counts and durations are per
            # frame; one launch of the kernel trace = launch_ms, frames_per_launch frames
            "launch": {"frames_per_launch": fpl, "launch_ms": round(avg_ms * (args.steps / n_launch), 4),
                       "timed_launches": n_launch,
                       "grid_blocks": s_get(dev, "grid_blocks"), "block": 64,
                       "blocks_per_cu_query": s_get(dev, "blocks_per_cu"),
                       "bvh_nodes": s_get(dev, "bvh_nodes"), "bvh_stack": s_get(dev, "bvh_stack"),
                       "group_spp": s_get(dev, "group_spp")},
            "image_mean": float(img.mean()),
        }
        rays = st_counts["camera_rays"] + st_counts["bounce_rays"] + st_counts["shadow_rays"]
        out["ray_casts_per_s_M"] = round(rays * frames * (world if weak else 1) / elapsed / 1e6, 1)
        # The rates a reader needs beside `value`: samples
        # actually traced (the footprint cull's samples excluded; a strong
        # split sums its ranks' culls), and one frame alone (no overlap with a
        # neighbouring frame: W*H*spp / single_frame_ms)
        culled = (sum(r[5] for r in per_rank) if (per_rank and not weak) else
                  st_counts["culled_samples"] * (world if weak else 1))
        out["traced_samples_per_s_M"] = round((W * H * SPP * (world if weak else 1) - culled) * frames / elapsed / 1e6, 1)
        out["single_frame_Mrays"] = None if single_ms is None else round(W * H * SPP / (single_ms * 1e-3) / 1e6, 1)
        if frame_batch is not None:
            out["one_frame_per_launch"] = frame_batch
        # the graded kernel fraction: the isolated launch's VALU-issue fraction
        vv = out["roofline"]["views"].get("valu")
        out["roofline"]["frac_kernel"] = vv.get("frac_isolated") if vv else None
        if per_rank is not None:
            out["per_rank"] = {"fields": ["kernel_ms", "resolve_ms", "exchange_ms", "pixels", "partial_bytes",
                                          "culled_samples"],
                               "ranks": per_rank}
        if xev or pex is not None:
            out["exchange_ms"] = round(xchg_ms, 4)
        if world > 1 and not weak:
            # the strong split's scaling inputs (ADVICE r5:
            # rate_1 from rank 0 alone, efficiency null when ranks share a GPU)
            out["single_gpu_value"] = None if rate1 is None else round(rate1, 1)
            out["efficiency"] = None if (rate1 is None or shared) else round(value / (world * rate1), 4)
            out["shared_device"] = shared
            out["exchange"] = ("pipelined: packed-tile gather + scatter of frame k queued behind its resolve, "
                               "overlapping frame k+1's render (render-slot streams)" if not pex.side else
                               "pipelined: packed-tile gather + scatter of frame k on a side stream behind an event, "
                               "overlapping frame k+1's render (double-buffered packed tiles)")
            if per_rank:
                kms = [r[0] for r in per_rank]
                out["kernel_ms_slowest_over_mean"] = round(max(kms) / max(1e-9, float(np.mean(kms))), 4)
        if multi is not None:
            out["companions"] = multi
        if world == 1 and not args.no_extras and workload == "c3" and not args.scene_dump:
            out["companions"] = companions(dev, local, stream, max(2, min(args.steps, 5)))
        out["dist"] = {"backend": backend if world > 1 else None,
                       "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                       "timeout_s": float(os.environ.get("PT_DIST_TIMEOUT", "120")) if world > 1 else None,
                       "value_knobs": knobs}
        if world == 1 and not args.no_cpu_baseline:
            try:
                dp = dump_path
                if dp is None:
                    from dsgpuraytracing_amd import scene_loader
                    os.makedirs(os.path.join(ROOT, "_scenes"), exist_ok=True)
                    dp = os.path.join(ROOT, "_scenes", f"bench_{workload}.ptd")
                    scene_loader.dump_dae(dae, W, H, dp, cam_info=cam, envmap=envmap)
                if dae is not None and os.access(REF_DRIVER, os.X_OK) and cam is None:
                    out["cpu_baseline"] = cpu_baseline_reference(dae, envmap)
                    # the reference at its published setting (readme.txt:1: -t 8)
                    out["cpu_baseline_published"] = cpu_baseline_reference(dae, envmap, budget_s=10.0, threads=8)
                else:  # the bit-identical restatement when the reference build is absent
                    out["cpu_baseline"] = cpu_baseline_port(dp)
                out["cpu_baseline_fair"] = cpu_baseline_port(dp, budget_s=10.0, rng_mode=1, threads=host_threads())
            except Exception as e:  # reported, never silently replaced
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)


def device_fingerprint(local: int) -> str:
    """This rank's GPU: host and device UUID (or ordinal): two ranks with the
    same fingerprint share one device (the one-GPU rehearsal)."""
    import socket

    import torch
    try:
        dev_id = str(torch.cuda.get_device_properties(local).uuid)
    except Exception:  # pragma: no cover - older torch without uuid
        dev_id = str(local)
    return f"{socket.gethostname()}:{dev_id}"


def single_gpu_rate(dev, tiles, w, h, spp, frame, stream, rank, backend, frames, warmup=2, fpl=1):
    """Collective.  The 1-GPU point of the strong-split curve: rank 0 renders
    the WHOLE frame `frames` times alone, back to back, behind a barrier (the
    other ranks wait in it, their GPUs idle), synchronised on both sides ->
    M samples/s, broadcast to every rank; with `fpl` frames per launch, as the
    N-GPU line renders its shares.  Also whether two ranks share a device
    (then the N-rank value is no scaling point: efficiency null)."""
    import torch
    import torch.distributed as dist

    fps = [None] * dist.get_world_size()
    dist.all_gather_object(fps, device_fingerprint(torch.cuda.current_device()))
    shared = len(set(fps)) < len(fps)
    dist.barrier()
    rate = torch.zeros(1, dtype=torch.float64, device="cpu" if backend == "gloo" else frame.device)
    if rank == 0:
        whole = np.asarray(tiles, dtype=np.int32).reshape(-1, 4)
        scratch = torch.empty_like(frame)
        def render(n):
            k = 0
            while k < n:
                m = min(max(1, fpl), n - k)
                if m == 1:
                    dev.render_tiles_device(whole, scratch.data_ptr(), stream)
                else:
                    dev.render_frames_device(whole, [scratch.data_ptr()] * m, [SEED] * m, stream)
                k += m

        render(warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        render(frames)
        torch.cuda.synchronize()
        rate.fill_(w * h * spp * frames / (time.perf_counter() - t0) / 1e6)
        del scratch
    dist.barrier()
    dist.broadcast(rate, src=0)
    return float(rate.item()), shared


def timed_max(el, backend, local):
    """Collective: the slowest rank's time of a region every rank timed."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([el], dtype=torch.float64, device="cpu" if backend == "gloo" else f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def multi_gpu_companions(local, rank, world, backend, StepGuard, PipelinedExchange, frames=5, warmup=2,
                         with_weak=True, split_tile=32, split_deal="diag", deal_block=0):
    """N > 1 companions (never `value`), same clock as the headline (barrier +
    synchronise on both sides of `frames` back-to-back frames, max over
    ranks):
      * c4_strong: BASELINE C4 (1080p, 256 spp, the multi-GPU config), its
        32x32 tiles dealt diagonally over the N GPUs, packed tiles gathered
        onto rank 0 behind each frame's resolve while the next frame renders (SURVEY.md
        §8(e)); efficiency against rank 0 rendering the whole frame alone;
        images bit-identical to 1 GPU (tests/test_dist.py,
        test_c4_fullsize_eight_way_split_bit_identical);
      * c3_weak: the headline frame as N disjoint 64-spp passes, one per GPU
        (sample indices 64r .. 64r+63; the counter RNG is keyed by the sample
        index), then ONE RCCL sum-reduce of the footprint's rows onto rank 0:
        a 64N-spp image; value = N*W*H*64*frames / time."""
    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    res = {}
    stream = torch.cuda.current_stream().cuda_stream
    wl = WORKLOADS["c4"]
    w, h, spp = wl["w"], wl["h"], wl["spp"]
    dae, envmap, cam = workload_scene(wl)
    sc = Scene.from_dae(dae, w, h, cam_info=cam, envmap=envmap)
    dev = Device(local)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(w, h, spp, DEPTH, NSL, SEED)
    frame = torch.zeros((h, w, 3), dtype=torch.float32, device=f"cuda:{local}")
    tiles = tile_fifo(w, h, split_tile)
    pex = PipelinedExchange(tiles, w, h, rank, world, frame.device, deal=split_deal, tile_size=split_tile,
                            deal_block=deal_block, **xchg_opts())
    mine = np.asarray(pex.mine, dtype=np.int32).reshape(-1, 4)
    guard = StepGuard()
    kf = [0]

    def step(timed=False, stats=False):
        k = kf[0]
        kf[0] += 1
        buf = pex.packed_for(k)
        guard.run(dev.render_tiles_device, mine, buf.data_ptr(), stream, packed=pex.ex.slot, out_floats=buf.numel(),
                  stats=stats)
        pex.exchange(k, frame, timed=timed)

    for _ in range(warmup):
        step()
    guard.check()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        step(timed=True)
    pex.drain()
    dist.barrier()
    torch.cuda.synchronize()
    el = timed_max(time.perf_counter() - t0, backend, local)
    guard.check()
    k_ms, _ = dev.launch_times(frames)
    step(stats=True)
    st = dev.stats()
    rate1, shared = single_gpu_rate(dev, tiles, w, h, spp, frame, stream, rank, backend, frames)
    mine_v = torch.tensor([float(np.mean(k_ms)), pex.exchange_ms(), float(np.sum(mine[:, 2] * mine[:, 3])),
                           float(st["partial_bytes"])],
                          dtype=torch.float64, device="cpu" if backend == "gloo" else f"cuda:{local}")
    allr = [torch.zeros_like(mine_v) for _ in range(world)]
    dist.all_gather(allr, mine_v)
    ranks = [[round(float(v), 4) for v in r.cpu().tolist()] for r in allr]
    kms = [r[0] for r in ranks]
    value = w * h * spp * frames / el / 1e6
    res["c4_strong"] = {
        "workload": wl["desc"] + f", one frame's tiles over {world} GPUs + one pipelined gather (strong)",
        "value": round(value, 1), "unit": "Mrays/s", "single_gpu_value": round(rate1, 1),
        "efficiency": None if shared else round(value / (world * rate1), 4), "shared_device": shared,
        "ms_per_frame": round(el / frames * 1e3, 3), "frames": frames, "scaling": "strong",
        "gather_bytes_per_rank": int(pex.ex.packed.numel() * 4),
        "kernel_ms_slowest_over_mean": round(max(kms) / max(1e-9, float(np.mean(kms))), 4),
        "per_rank": {"fields": ["kernel_ms", "exchange_ms", "pixels", "partial_bytes"], "ranks": ranks},
        "image_mean": float(frame.mean().item()) if rank == 0 else None}
    dev.close()
    del frame, pex
    if with_weak:
        res["c3_weak"] = weak_companion(local, rank, world, backend, StepGuard, frames, warmup)
    return res


def weak_companion(local, rank, world, backend, StepGuard, frames, warmup=2):
    """c3_weak (see multi_gpu_companions)."""
    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    wl = WORKLOADS["c3"]
    w, h, spp = wl["w"], wl["h"], wl["spp"]
    dae, envmap, cam = workload_scene(wl)
    sc = Scene.from_dae(dae, w, h, cam_info=cam, envmap=envmap)
    dev = Device(local)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(w, h, spp, DEPTH, NSL, SEED, sample_base=spp * rank)
    stream = torch.cuda.current_stream().cuda_stream
    frame = torch.zeros((h, w, 3), dtype=torch.float32, device=f"cuda:{local}")
    whole = np.asarray(tile_fifo(w, h), dtype=np.int32).reshape(-1, 4)
    guard = StepGuard()
    guard.run(dev.render_tiles_device, whole, frame.data_ptr(), stream, stats=True)
    st = guard.run(dev.stats)
    guard.check()
    # rows outside the screen footprint are 0 in every pass: the reduce carries the footprint's rows only
    y0, y1 = st["footprint"][1], st["footprint"][3]
    rows = frame[y0:y1 + 1] if y1 >= y0 else frame[:0]
    xev = []

    def step(timed=False):
        guard.run(dev.render_tiles_device, whole, frame.data_ptr(), stream)
        if rows.numel() == 0:
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        if backend == "gloo":  # host staging (one-GPU rehearsals)
            hb = rows.cpu()
            dist.reduce(hb, dst=0)
            if rank == 0:
                rows.copy_(hb)
        else:
            dist.reduce(rows, dst=0)
        if rank == 0:
            rows.mul_(1.0 / world)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        if timed:
            xev.append((e0, e1))

    for _ in range(warmup):
        step()
    guard.check()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        step(timed=True)
    dist.barrier()
    torch.cuda.synchronize()
    el = timed_max(time.perf_counter() - t0, backend, local)
    guard.check()
    out = {"workload": wl["desc"] + f", one 64-spp pass per GPU over disjoint sample indices + one RCCL reduce "
                                    f"(a {spp * world}-spp image; weak)",
           "value": round(world * w * h * spp * frames / el / 1e6, 1), "unit": "Mrays/s",
           "ms_per_frame": round(el / frames * 1e3, 3), "frames": frames, "scaling": "weak",
           "reduce_bytes_per_rank": int(rows.numel() * 4),
           "reduce_ms": round(float(np.mean([a.elapsed_time(b) for a, b in xev])), 4) if xev else 0.0,
           "image_mean": float(frame.mean().item()) if rank == 0 else None}
    dev.close()
    return out


def bvh_desc(lbvh=False):
    """The render tree a run traces (pt_api.cpp upload_impl)."""
    b = os.environ.get("PT_BVH_BUILD")
    if lbvh:
        return "gpu-lbvh via pt_upload_scene_lbvh (Karras + treelet restructuring, device-built)"
    if b == "ref":
        return "the caller's reference tree (BVHAccel, host)"
    if b == "sah":
        return "own binned SAH, 128 bins, C_isect 1 (host)"
    return ("own GPU-built tree: Karras LBVH + %s treelet-restructuring passes (device)"
            % os.environ.get("PT_LBVH_PASSES", "3"))


def s_get(dev, key):
    return dev.stats().get(key)


def companions(dev0, local, stream, frames):
    """One-GPU companion numbers printed beside the C3 headline (not `value`):
      * c3_framed: C3 through a camera that frames the box interior, so every
        sample is traced (the headline's default camera leaves ~75% of the
        frame outside the scene's footprint);
      * c4_single_gpu: BASELINE C4 on this one GPU, the 1-GPU point of the
        multi-GPU (C4, strong) scaling curve;
      * c5_single_gpu: BASELINE C5 (glass/mirror proxy + environment light)
        on this one GPU;
      * c5big_single_gpu: C5 at BASELINE's "~1M tris" scale (the sub3 proxy,
        1.83 M triangles: the one workload whose scene leaves the L2s), with
        its own PMC roofline (profiles/<round>/c5big_summary.json);
      * c3_host_sah: the headline workload over the host binned-SAH tree
        (PT_BVH_BUILD=sah) instead of the default GPU-built tree;
      * c3_per_tile / c3_per_tile_sync: the headline frame driven through the
        reference's literal seam -- 8 worker threads calling raytrace_tile
        once per 32x32 tile (1,024 calls, pathtracer.cpp:585-621) through one
        context, as INTEGRATION.md's adapter does -- asynchronously
        (pt_tile_submit: tiles batched into launches, completed into the
        host sampleBuffer + toColor'd frameBuffer by a completion thread) and with
        one synchronous pt_render_tiles launch per tile.  Host output
        included (PCIe), so these are never `value`."""
    import torch

    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    res = {}
    names = {"c3f": "c3_framed", "c4": "c4_single_gpu", "c5": "c5_single_gpu", "c5big": "c5big_single_gpu",
             "c3": "c3_host_sah"}
    for name in ("c3f", "c4", "c5", "c5big", "c3"):
        wl = WORKLOADS[name]
        host_sah = name == "c3"
        dae, envmap, cam = workload_scene(wl)
        sc = Scene.from_dae(dae, wl["w"], wl["h"], cam_info=cam, envmap=envmap)
        dev = Device(local)
        old = os.environ.get("PT_BVH_BUILD")
        if host_sah:
            os.environ["PT_BVH_BUILD"] = "sah"
        t_up = time.perf_counter()
        dev.upload_scene(sc)
        t_up = time.perf_counter() - t_up
        bvh = bvh_desc()
        if host_sah:
            if old is None:
                del os.environ["PT_BVH_BUILD"]
            else:
                os.environ["PT_BVH_BUILD"] = old
        dev.set_camera(sc.camera)
        dev.set_params(wl["w"], wl["h"], wl["spp"], DEPTH, NSL, SEED)
        tl = np.asarray(tile_fifo(wl["w"], wl["h"]), np.int32)
        fr = torch.zeros((wl["h"], wl["w"], 3), dtype=torch.float32, device=f"cuda:{local}")
        dev.render_tiles_device(tl, fr.data_ptr(), stream)
        dev.render_tiles_device(tl, fr.data_ptr(), stream, stats=True)
        st = dev.stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            dev.render_tiles_device(tl, fr.data_ptr(), stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        k, _ = dev.launch_times(frames)
        rays = st["camera_rays"] + st["bounce_rays"] + st["shadow_rays"]
        res[names[name]] = {
            "workload": wl["desc"], "value": round(wl["w"] * wl["h"] * wl["spp"] * frames / el / 1e6, 1),
            "unit": "Mrays/s", "ms_per_step": round(el / frames * 1e3, 3), "kernel_ms": round(float(np.mean(k)), 3),
            "frames": frames, "culled_samples": st["culled_samples"],
            "ray_casts_per_s_M": round(rays * frames / el / 1e6, 1), "upload_s": round(t_up, 4),
            "bvh": bvh}
        if name == "c5big":  # its own roofline: the counts of profiles/<round>/c5big_summary.json
            dev.render_tiles_device(tl, fr.data_ptr(), stream, stats="ref")
            st_ref = dev.stats()
            iso = []
            for _ in range(2):  # lone, synchronised frames: the kernel's own duration
                torch.cuda.synchronize()
                dev.render_tiles_device(tl, fr.data_ptr(), stream)
                torch.cuda.synchronize()
                iso.append(dev.launch_times(1)[0][0])
            res[names[name]]["roofline"] = roofline(name, el / frames * 1e3, algorithmic_bytes(st_ref),
                                                    isolated_ms=float(np.median(iso)), pipelined_ms=float(np.mean(k)),
                                                    lib_sha=lib_sha256(), kernel_sha=kernel_sha256())
        dev.close()
        del fr
    res.update(per_tile_companions(local))
    return res


def per_tile_companions(local, threads=8):
    from dsgpuraytracing_amd.pathtracer import PathTracer, Scene
    wl = WORKLOADS["c3"]
    dae, envmap, cam = workload_scene(wl)
    sc = Scene.from_dae(dae, wl["w"], wl["h"], cam_info=cam, envmap=envmap)
    out = {}
    for name, asynchronous, frames in (("c3_per_tile", True, 3), ("c3_per_tile_sync", False, 1)):
        pt = PathTracer(ns_aa=wl["spp"], max_ray_depth=DEPTH, ns_area_light=NSL, seed=SEED, device=local)
        pt.set_frame_size(wl["w"], wl["h"])
        pt.set_camera(sc.camera)
        pt.set_scene(sc)
        pt.render_tile_workers(num_threads=threads, asynchronous=asynchronous)  # warm-up frame
        t0 = time.perf_counter()
        for _ in range(frames):
            pt.render_tile_workers(num_threads=threads, asynchronous=asynchronous)
        el = (time.perf_counter() - t0) / frames
        out[name] = {"workload": wl["desc"] + f", {threads} worker threads x 1,024 raytrace_tile calls "
                                              f"({'pt_tile_submit, batched' if asynchronous else 'pt_render_tiles, one launch each'})",
                     "value": round(wl["w"] * wl["h"] * wl["spp"] / el / 1e6, 1), "unit": "Mrays/s",
                     "ms_per_frame": round(el * 1e3, 3), "frames": frames, "threads": threads,
                     "host_output": "sampleBuffer + toColor frameBuffer (PCIe-inclusive)"}
        pt._device().close()
    out["c3_per_tile_native"] = seam_native(wl, dae, cam, threads)
    return out


def seam_native(wl, dae, cam, threads, frames=3):
    """The same per-tile seam driven from C++ (tools/seam_bench.cpp: 8
    std::thread workers, one context, a mutex around raytrace_tile), so the
    seam is timed without the Python adapter; also the whole frame as one
    pt_render_tiles call + pt_to_color with host output, and a bit-for-bit
    check of both seams against it.  A child process: this process's own
    contexts are closed first."""
    import subprocess
    exe = os.path.join(ROOT, "dsgpuraytracing_amd", "seam_bench")
    if cam is not None or not os.path.exists(exe):
        return {"skipped": "no seam_bench binary" if cam is None else "camera file not supported"}
    r = subprocess.run([exe, dae, str(wl["w"]), str(wl["h"]), str(wl["spp"]), str(threads), str(frames)],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    if r.returncode not in (0, 3):
        raise RuntimeError(f"seam_bench failed ({r.returncode}): {r.stderr.decode(errors='replace')[-400:]}")
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    res["workload"] = wl["desc"] + f", C++ driver, {threads} std::thread workers"
    res["unit"] = "Mrays/s"
    res["frames"] = frames
    return res


if __name__ == "__main__":
    main()
