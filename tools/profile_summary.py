"""Summarise a rocprofv3 profiling session of bench.py into profiles/<round>/.

Reads the passes written by tools/profile_session.sh under gpurun_out/prof/:
  kt/     --kernel-trace --stats      (per-kernel average duration, render pipeline on:
                                       consecutive launches overlap)
  kt_iso/ --kernel-trace --stats      with PT_PIPELINE=0 (every launch alone: the kernel's
                                       own duration, bench.py's isolated_kernel_ms)
  fetch/  --pmc FETCH_SIZE            (KB; doubled per MI355X_MICROARCH.md §HBM)
  write/  --pmc WRITE_SIZE            (KB)
  sq/     --pmc SQ_*                  (quad-cycle units for *_CYCLES / WAIT / ACTIVE)
  tcc/    --pmc TCC_HIT_sum TCC_MISS_sum
and writes <out>/<workload>_kernel_stats.csv and <out>/<workload>_summary.json
(bench.py's roofline reads the newest round's summary of its workload), stamped
with the sha256 of the libptgpu.so the passes ran (bench.py reports pmc_stale
when it loads a different one).  The PMC passes run with PT_PIPELINE=0.
Frame batches (round 6): when bench.py's timed launches render F frames each
(--frames-per-launch; the C3 line renders 8), pass F: the timed kernel is then
the frame-batch instantiation (MF), and every count of the summary -- HBM
bytes, SQ / TCC counters, the durations' per-frame fields -- is per FRAME (the
per-launch count / F), which is what bench.py's roofline divides by its
per-frame interval; `avg_ms` / `isolated_avg_ms` stay per launch (they must
agree with the kernel-trace files beside them).
Usage: python tools/profile_summary.py <workload> <out_dir> [prof_dir] [lib] [frames_per_launch]
"""
import collections
import csv
import hashlib
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dsgpuraytracing_amd.elfsha import kernel_sha256  # noqa: E402

# render_kernel<STATS, DBG, BIN, ENV, GTAB[, TRI]>: the timed launch of each workload (prefix:
# the triangle-only and the mixed instantiation; one bench run launches one of them)
KERNELS = {"c5": "render_kernel<false, false, false, true, false", "c5big": "render_kernel<false, false, false, true, false"}
KERNEL = "render_kernel<false, false, false, false, false"


FPL = 1  # frames per timed launch


def timed(name):
    """The workload's timed render launch: the kernel prefix, and the
    frame-batch instantiation (last template argument MF = true) exactly when
    the timed launches render several frames each (the profiled process also
    launches the other one: single frames, per-launch companions)."""
    return KERNEL in name and ((", true>(" in name) == (FPL > 1))


def _pmc(path):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if timed(r["Kernel_Name"]):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    global KERNEL, FPL
    workload, out = sys.argv[1], sys.argv[2]
    FPL = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    KERNEL = KERNELS.get(workload, KERNEL)
    prof = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/prof"
    lib = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "dsgpuraytracing_amd", "libptgpu.so")
    os.makedirs(out, exist_ok=True)
    ks = os.path.join(prof, "kt", "kt_kernel_stats.csv")
    shutil.copy(ks, os.path.join(out, f"{workload}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(ks))}
    render = next(v for k, v in stats.items() if timed(k))
    resolve = next((v for k, v in stats.items() if "resolve_kernel" in k), None)
    iso = None
    ksi = os.path.join(prof, "kt_iso", "kt_iso_kernel_stats.csv")
    if os.path.exists(ksi):
        shutil.copy(ksi, os.path.join(out, f"{workload}_kernel_stats_isolated.csv"))
        iso = next(v for k, v in {r["Name"]: r for r in csv.DictReader(open(ksi))}.items() if timed(k))
    def per_frame(d):  # a batch launch's counts per frame
        return {k: v / FPL for k, v in d.items()}

    fetch = per_frame(_pmc(os.path.join(prof, "fetch", "fetch_counter_collection.csv")))
    write = per_frame(_pmc(os.path.join(prof, "write", "write_counter_collection.csv")))
    sq = per_frame(_pmc(os.path.join(prof, "sq", "sq_counter_collection.csv")))
    tcc = per_frame(_pmc(os.path.join(prof, "tcc", "tcc_counter_collection.csv")))
    for name, d in (("fetch", fetch), ("write", write), ("sq", sq), ("tcc", tcc)):
        src = os.path.join(prof, name, f"{name}_counter_collection.csv")
        if os.path.exists(src):
            rows = [r for r in csv.DictReader(open(src)) if timed(r["Kernel_Name"])]
            with open(os.path.join(out, f"{workload}_pmc_{name}.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
    avg_ns = float(render["AverageNs"])
    s = {
        "workload": workload,
        "kernel": KERNEL,
        "kernel_name": next(k for k in stats if timed(k)),
        "frames_per_launch": FPL,
        "counts_per": "frame",
        "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
        "kernel_sha256": kernel_sha256(lib),
        "calls": int(render["Calls"]),
        "avg_ms": avg_ns / 1e6,
        "isolated_avg_ms": float(iso["AverageNs"]) / 1e6 if iso else None,
        "resolve_avg_ms": float(resolve["AverageNs"]) / 1e6 if resolve else None,
    }
    if FPL > 1:
        s["avg_ms_per_frame"] = s["avg_ms"] / FPL
        s["isolated_avg_ms_per_frame"] = s["isolated_avg_ms"] / FPL if iso else None
    if iso:  # utilisation over the kernel's own duration, not an overlapped span
        avg_ns = float(iso["AverageNs"])
    avg_ns /= FPL  # (per frame, as the counts)
    if "FETCH_SIZE" in fetch and "WRITE_SIZE" in write:
        s["fetch_size_kb"] = fetch["FETCH_SIZE"]
        s["write_size_kb"] = write["WRITE_SIZE"]
        s["hbm_bytes_per_launch"] = (2.0 * fetch["FETCH_SIZE"] + write["WRITE_SIZE"]) * 1024.0
        s["hbm_gbs"] = s["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
    if sq:
        cyc = avg_ns * 1e-9 * 2.4e9
        s["sq"] = sq
        if "SQ_INSTS_VALU" in sq:  # 256 CUs, 2 wave64 VALU issues per CU-cycle (4 SIMD-32)
            s["valu_issue_util"] = sq["SQ_INSTS_VALU"] / (256 * 2 * cyc)
        if "SQ_WAVE_CYCLES" in sq:
            wc = sq["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in sq:
                    s[k.lower() + "_frac"] = sq[k] / wc
    if tcc:
        s["tcc"] = tcc
        if "TCC_HIT_sum" in tcc:
            s["l2_hit_rate"] = tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"])
    with open(os.path.join(out, f"{workload}_summary.json"), "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps(s, indent=1))


if __name__ == "__main__":
    main()
