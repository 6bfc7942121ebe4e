"""Per-launch averages of the render kernel's extra PMC passes
(tools/profile_deep.sh -> gpurun_out/prof/{sq2,sq3,tcp,tcp2,ta}/) and the
derived memory-pipe figures.  The kernel's isolated duration comes from the
profile summary of the same workload (profiles/<round>/<wl>_summary.json).
Usage: python tools/deep_summary.py <workload> <summary.json> [prof_dir]"""
import collections
import csv
import json
import os
import sys

KERNELS = {"c5": "render_kernel<false, false, false, true, false"}
wl, summ = sys.argv[1], sys.argv[2]
prof = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/prof"
K = KERNELS.get(wl, "render_kernel<false, false, false, false, false")
vals = {}
for name in ("sq2", "sq3", "tcp", "tcp2", "ta"):
    p = os.path.join(prof, name, f"{name}_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if K in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    vals.update({k: sum(v) / len(v) for k, v in agg.items()})
s = json.load(open(summ))
ms = s.get("isolated_avg_ms") or s["avg_ms"]
cu_cycles = 256 * ms * 1e-3 * 2.4e9  # CU-cycles of one launch at 2.4 GHz
out = {"workload": wl, "kernel_ms": ms, "counters": vals}
if "TA_TA_BUSY_sum" in vals:
    out["ta_busy_frac"] = vals["TA_TA_BUSY_sum"] / cu_cycles
if "SQ_INSTS_VMEM_RD" in vals:
    out["vmem_rd_per_launch"] = vals["SQ_INSTS_VMEM_RD"]
    if "SQ_INSTS_VALU" in s.get("sq", {}):
        out["valu_per_vmem_rd"] = s["sq"]["SQ_INSTS_VALU"] / vals["SQ_INSTS_VMEM_RD"]
if "TCP_TOTAL_CACHE_ACCESSES_sum" in vals and "TCP_TCC_READ_REQ_sum" in vals:
    out["l1_hit_rate"] = 1.0 - vals["TCP_TCC_READ_REQ_sum"] / max(1.0, vals["TCP_TOTAL_CACHE_ACCESSES_sum"])
if "TCP_TCC_READ_REQ_LATENCY_sum" in vals and "TCP_TCC_READ_REQ_sum" in vals:
    out["l1_miss_latency_cycles"] = vals["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1.0, vals["TCP_TCC_READ_REQ_sum"])
for k in ("TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TCP_TCP_TA_DATA_STALL_CYCLES_sum"):
    if k in vals:
        out[k.lower().replace("_sum", "") + "_frac"] = vals[k] / cu_cycles
print(json.dumps(out, indent=1))
