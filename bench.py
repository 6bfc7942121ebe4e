#!/usr/bin/env python3
"""Benchmark of the path-tracing hot path on MI355X.

Metric (BASELINE.json): "Mrays/sec + wall-clock render time, CBdragon 1024x1024
@ 64 spp".  A "step" is one full-frame render (every 32x32 tile of the
reference's FIFO) of the C3 workload: 1024x1024, 64 spp, max_ray_depth 4,
ns_area_light 1 (readme.txt:1 settings) on the CBdragon proxy CBbunny_sub1
(114,316 triangles; CBdragon.dae is absent).
Mrays/s = W*H*spp*frames / seconds / 1e6 (primary path samples, the unit of the
reference's "Primary (M ray/s)" column); scene load / BVH build / upload are
outside the timed region, as in the reference's timers.

N > 1 (one process per GPU, torchrun), default --scaling weak: the path
partitions into independent (pixel, sample) units, and every GPU renders one
64-spp pass of the whole C3 frame with its own sample range (rank r: sample
indices 64r .. 64r+63, pt_params.sample_base), i.e. exactly the 1-GPU
workload; one RCCL sum-reduce over xGMI assembles the 64N-spp image on rank 0
(the framebuffer exchange of SURVEY.md §8(e)).  value = N * W*H*64 / max-rank
time, "scaling": "weak".  --scaling strong splits ONE 64-spp frame instead:
ranks render interleaved 32x32 tiles into packed tile buffers
(PT_FLAG_PACKED) that one RCCL gather brings to rank 0 (bit-identical to the
1-GPU image); value = W*H*64 / max-rank time.  The exchange is inside the
timed region in both modes.
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

# BASELINE.json configs; C3 is the headline (default).
WORKLOADS = {
    "c1": dict(scene="c1", w=256, h=256, spp=1, desc="C1 CBspheres_lambertian 256x256 1spp -m 4 -l 1"),
    "c2": dict(scene="c1", w=512, h=512, spp=16, desc="C2 CBspheres_lambertian 512x512 16spp -m 4 -l 1"),
    "c3": dict(scene="sub1", w=1024, h=1024, spp=64,
               desc="C3 CBbunny_sub1 (114,316 tris; CBdragon proxy) 1024x1024 64spp -m 4 -l 1"),
    "c4": dict(scene="sub1", w=1920, h=1080, spp=256,
               desc="C4 CBbunny_sub1 (CBdragon proxy) 1920x1080 256spp -m 4 -l 1, tiles over N GPUs"),
    "c5": dict(scene="c5", w=1920, h=1080, spp=512,
               desc="C5 CBbunny_sub2_c5 (457,228 tris, glass bunny + mirror sphere; CBlucy proxy) + synthetic "
                    "512x256 environment light, 1920x1080 512spp -m 4 -l 1, tiles over N GPUs"),
}
W, H, SPP, DEPTH, NSL, SEED = 1024, 1024, 64, 4, 1, 1
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(st: dict) -> float:
    """SURVEY.md §8(d) reference-layout cost model: 64 B per BVH node visit,
    48 B per triangle test, 16 B per sphere test, 4 B per leaf primitive index,
    36 B per hit (vertex normals), 12 B per pixel written."""
    prim = st["tri_tests"] + st["sphere_tests"]
    return (64.0 * st["node_visits"] + 48.0 * st["tri_tests"] + 16.0 * st["sphere_tests"] + 4.0 * prim
            + 36.0 * st["ext_hits"] + 12.0 * st["pixels"])


def measured_traffic(workload: str):
    """HBM bytes per launch of the render kernel on this workload, from the
    rocprofv3 PMC passes committed under profiles/ (tools/profile_summary.py:
    FETCH_SIZE doubled per the gfx950 correction of MI355X_MICROARCH.md §HBM,
    + WRITE_SIZE; KB -> bytes).  None when no summary for this workload is
    committed."""
    p = os.path.join(ROOT, "profiles", "latest_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch") if d.get("workload") == workload else None
    except (OSError, ValueError):
        return None


def measured_pmc(workload: str):
    """Issue/latency view of the render kernel from the committed PMC summary
    (informational: the kernel is latency- and issue-bound, not HBM-bound)."""
    try:
        with open(os.path.join(ROOT, "profiles", "latest_traffic.json")) as f:
            src = json.load(f)["source"]
        with open(os.path.join(ROOT, src)) as f:
            d = json.load(f)
        if d.get("workload") != workload:
            return None
        keys = ("avg_ms", "hbm_gbs", "l2_hit_rate", "valu_issue_util", "sq_wait_any_frac", "sq_wait_inst_any_frac",
                "sq_active_inst_any_frac")
        return {k: (round(d[k], 4) if isinstance(d.get(k), float) else d.get(k)) for k in keys} | {"source": src}
    except (OSError, ValueError, KeyError):
        return None


REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")


def cpu_baseline_reference(dae: str, envmap, budget_s: float = 15.0) -> dict:
    """The reference's OWN CPU path (oracle/_ref/ref_driver, compiled from
    /root/reference/src by oracle/ref/Makefile; it travels to the GPU box with
    the tree) timed on this host: PathTracer::raytrace_tile (pathtracer.cpp:
    585-611) on every k-th 32x32 tile of the frame's FIFO, on one thread with
    glibc rand() as shipped (== its -t 1 setting, its fastest: the shared rand()
    lock makes it anti-scale with threads), k sized from a calibration run so
    the sample takes about budget_s.  Scene load and BVH build are excluded,
    as in the reference's own timer."""
    import math
    import subprocess

    ntx = (W + 31) // 32
    ntiles = ntx * ((H + 31) // 32)

    def coprime(k):  # strides sharing a factor with the row length sample columns, not the frame
        while k > 1 and math.gcd(k, ntx) != 1:
            k += 1
        return k

    def run(begin, stride):
        cmd = [REF_DRIVER, dae, "--mode", "tiles", "-w", str(W), "-h", str(H), "-s", str(SPP), "-m", str(DEPTH),
               "-l", str(NSL), "--seed", str(SEED), "--tile-begin", str(begin), "--tile-stride", str(stride)]
        if envmap:
            cmd += ["--envmap", envmap]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=600, check=True)
        return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])

    cal = coprime(max(1, ntiles // 12))
    c = run(cal // 2, cal)
    per_tile = max(c["render_s"], 1e-4) / max(1, c["tiles"])
    step = coprime(max(1, int(round(ntiles * per_tile / budget_s))))
    m = run(step // 2, step)
    return {"value": m["pixels"] * SPP / m["render_s"] / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "reference",
            "sample": f"every {step}th 32x32 tile of the {W}x{H} frame ({m['pixels']} px, uniform) at {SPP} spp, "
                      f"-m {DEPTH} -l {NSL}: the reference's PathTracer::raytrace_tile built from its own sources "
                      f"(oracle/_ref/ref_driver --mode tiles), one thread, glibc rand() as shipped (its -t 1), "
                      f"{m['render_s']:.1f} s of rendering"}


def cpu_baseline(scene_dump: str, budget_s: float = 12.0) -> dict:
    """Reference CPU algorithm (oracle/restate.cpp, bit-identical to the
    reference binary at -t 1: glibc rand, one thread) timed on this host on a
    bounded, UNIFORM sample of the same workload: every k-th tile of the 32x32
    tile FIFO at the full spp, k sized from a 16-tile calibration so the sample
    takes about budget_s (scene load excluded)."""
    from tests.oracle_helpers import Restatement
    rs = Restatement()
    ntx = (W + 31) // 32
    ntiles = ntx * ((H + 31) // 32)

    def tiles_px(begin, stride):
        px = 0
        for ti in range(begin, ntiles, stride):
            tx, ty = (ti % ntx) * 32, (ti // ntx) * 32
            px += (min(W, tx + 32) - tx) * (min(H, ty + 32) - ty)
        return px

    import math

    def coprime(k):  # strides sharing a factor with the row length sample columns, not the frame
        while k > 1 and math.gcd(k, ntx) != 1:
            k += 1
        return k

    cal = coprime(max(1, ntiles // 16))
    _, _, t_cal = rs.render_strided(scene_dump, W, H, SPP, DEPTH, NSL, SEED, rng_mode=0, tile_begin=cal // 2,
                                    tile_stride=cal)
    per_tile = max(t_cal, 1e-4) / len(range(cal // 2, ntiles, cal))
    step = coprime(max(1, int(round(ntiles * per_tile / budget_s))))
    _, _, secs = rs.render_strided(scene_dump, W, H, SPP, DEPTH, NSL, SEED, rng_mode=0, tile_begin=step // 2,
                                   tile_stride=step)
    px = tiles_px(step // 2, step)
    return {"value": px * SPP / secs / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"every {step}th 32x32 tile of the {W}x{H} frame ({px} px, uniform) at {SPP} spp, -m {DEPTH} "
                      f"-l {NSL}, oracle/restate.cpp glibc-rand mode (== reference -t 1), {secs:.1f} s of rendering"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene-dump", default=None, help="PTDUMP scene instead of the native .dae loader")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--lbvh", action="store_true", help="build the BVH on the GPU (pt_upload_scene_lbvh)")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="diagnostic: render only one rank's share of an N-GPU split on this one GPU")
    ap.add_argument("--emulate-rank", type=int, default=0, help="the rank --emulate-shard renders")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = one 64-spp pass of the whole frame per GPU (sample split); "
                         "strong = one frame's tiles split across the GPUs")
    args = ap.parse_args()
    global W, H, SPP
    wl = WORKLOADS[args.workload]
    W, H, SPP = wl["w"], wl["h"], wl["spp"]

    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.dist import TileExchange, init_from_env, shard_tiles
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

    from dsgpuraytracing_amd import scenes
    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo

    t_load = time.perf_counter()
    dae, envmap = None, None
    if args.scene_dump:
        scene = Scene.from_dump(args.scene_dump)
        dump_path = args.scene_dump
    else:
        if wl["scene"] == "sub1":
            dae = scenes.proxy_path(1)
        elif wl["scene"] == "c5":
            dae, envmap = scenes.c5_path(2), scenes.c5_envmap_path()
        else:
            dae = scenes.C1_DAE
        scene = Scene.from_dae(dae, W, H, envmap=envmap)
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

    tiles = tile_fifo(W, H)
    frame = torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream().cuda_stream

    # strong: this rank's share of the tiles; weak (and one GPU): every tile
    mine_arr = np.asarray(tiles if weak else shard_tiles(tiles, rank, world), dtype=np.int32).reshape(-1, 4)
    if args.emulate_shard > 1:
        mine_arr = np.asarray(shard_tiles(tiles, args.emulate_rank, args.emulate_shard),
                              dtype=np.int32).reshape(-1, 4)
    ex = TileExchange(tiles, W, H, rank, world, frame.device) if world > 1 and not weak else None
    if ex is not None:
        mine_arr = np.asarray(ex.mine, dtype=np.int32).reshape(-1, 4)

    def reduce_passes():  # weak: sum the N passes onto rank 0, mean over 64N samples
        if backend == "gloo":  # host staging (one-GPU rehearsals)
            h = frame.cpu()
            dist.reduce(h, dst=0)
            if rank == 0:
                frame.copy_(h)
        else:
            dist.reduce(frame, dst=0)
        if rank == 0:
            frame.mul_(1.0 / world)

    def step(stats=False):
        if ex is None:  # the whole tile FIFO straight into the frame (one GPU, or this rank's pass)
            dev.render_tiles_device(mine_arr, frame.data_ptr(), stream, stats=stats)
            if weak:
                reduce_passes()
        else:  # this rank's tiles into its packed buffer, then one gather onto rank 0
            dev.render_tiles_device(mine_arr, ex.packed.data_ptr(), stream, stats=stats, packed=True)
            ex.exchange(frame)
        return dev.stats() if stats else None

    # counters for the roofline's algorithmic bytes: the reference's binary BVH
    # (SURVEY.md §8(d) cost model); and the launch's own counters (4-wide BVH)
    st_counts = step(stats="ref")
    st_perf = step(stats=True)
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):  # asynchronous: nothing waits on the GPU inside a step
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # HIP events recorded around every launch on its stream (the timed ones)
    kernel_ms, resolve_ms = dev.launch_times(args.steps)
    s = dev.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    host_ms = None
    if world == 1:  # the drop-in pt_render_tiles path: output copied to a host buffer (PCIe-inclusive)
        host = np.zeros((H, W, 3), np.float32)
        dev.render_tiles(mine_arr, host)
        t0h = time.perf_counter()
        for _ in range(2):
            dev.render_tiles(mine_arr, host)
        host_ms = (time.perf_counter() - t0h) / 2 * 1e3
    if rank == 0:
        frames = args.steps
        value = W * H * SPP * frames * (world if weak else 1) / elapsed / 1e6
        if args.emulate_shard > 1:
            value = float(np.sum(mine_arr[:, 2] * mine_arr[:, 3])) * SPP * frames / elapsed / 1e6
        bytes_launch = algorithmic_bytes(st_counts)
        avg_ms = float(np.mean(kernel_ms))
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        img = frame.float().cpu().numpy()
        out = {
            "metric": "Mrays/sec + wall-clock render time, CBdragon 1024x1024 @ 64 spp"
                      if args.workload == "c3" else f"Mrays/sec + wall-clock render time, {wl['desc']}",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / frames * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": {"c5": "synthetic: deterministic CBbunny_sub2 glass/mirror proxy for the missing CBlucy.dae + "
                           "seeded 512x256 environment map (SURVEY §8(d))",
                     "c1": "CBspheres_lambertian.dae from the reference", "c2": "CBspheres_lambertian.dae from the reference"
                     }.get(args.workload,
                           "synthetic: deterministic CBbunny_sub1 proxy for the missing CBdragon.dae (SURVEY §8(d))"),
            "config": {"workload": wl["desc"] + ", default camera",
                       "width": W, "height": H, "spp": SPP, "max_ray_depth": DEPTH, "ns_area_light": NSL,
                       "spp_total": SPP * world if weak else SPP,
                       "parallelism": (f"samples{world}" if weak else f"tiles{world}") if world > 1 else "single",
                       "render_time_s": round(elapsed / frames, 4), "scene_load_s": round(t_load, 3),
                       "bvh": "gpu-lbvh" if args.lbvh else "reference-sah (host)",
                       "upload_s": round(t_up, 4),
                       "host_output_ms_per_frame": None if host_ms is None else round(host_ms, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": measured_traffic(args.workload),
                         "kernel": "render_kernel<false>", "kernel_ms": round(avg_ms, 3),
                         "resolve_ms": round(float(np.mean(resolve_ms)), 4),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "pmc": measured_pmc(args.workload)},
            "counters": {k: st_counts[k] for k in ("camera_rays", "bounce_rays", "shadow_rays", "node_visits",
                                                   "tri_tests", "sphere_tests", "ext_hits", "culled_samples")},
            "launch_counters": {k: st_perf[k] for k in ("node_visits", "tri_tests", "sphere_tests", "wave_trav_steps",
                                                        "leaf_steps", "wave_rounds", "queue_atomics", "shade_clocks",
                                                        "hitshade_clocks", "trav_clocks", "max_wave_clocks",
                                                        "wave_wall_sum", "wave_wall_max", "section_clocks", "wave_span",
                                                        "lane_iters")},
            "launch": {"grid_blocks": s["grid_blocks"], "block": 64, "blocks_per_cu_query": s["blocks_per_cu"],
                       "bvh_nodes": s["bvh_nodes"], "bvh_stack": s["bvh_stack"]},
            "image_mean": float(img.mean()),
        }
        rays = st_counts["camera_rays"] + st_counts["bounce_rays"] + st_counts["shadow_rays"]
        if world == 1:
            out["ray_casts_per_s_M"] = round(rays * frames / elapsed / 1e6, 1)
        if world == 1 and not args.no_cpu_baseline:
            try:
                dp = dump_path
                if dp is None:
                    from dsgpuraytracing_amd import scene_loader
                    dp = os.path.join(ROOT, "_scenes", f"bench_{args.workload}.ptd")
                    scene_loader.dump_dae(dae, W, H, dp, envmap=envmap)
                if dae is not None and os.access(REF_DRIVER, os.X_OK):
                    out["cpu_baseline"] = cpu_baseline_reference(dae, envmap)
                else:  # the bit-identical restatement when the reference build is absent
                    out["cpu_baseline"] = cpu_baseline(dp)
            except Exception as e:  # reported, never silently replaced
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
