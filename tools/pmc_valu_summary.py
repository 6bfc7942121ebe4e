#!/usr/bin/env python3
"""Per-launch averages of the render kernel's SQ counters for each arm of
tools/pmc_valu.sh.  Usage: python tools/pmc_valu_summary.py <dir> <workload>"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = {"c5": "render_kernel<false, false, false, true, false",
          "c5big": "render_kernel<false, false, false, true, false"}


def main():
    d, wl = sys.argv[1], sys.argv[2]
    kern = KERNEL.get(wl, "render_kernel<false, false, false, false, false")
    for arm in sorted(os.listdir(d)):
        files = glob.glob(os.path.join(d, arm, "**", "*counter_collection.csv"), recursive=True)
        agg = collections.defaultdict(list)
        for f in files:
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        avg = {k: sum(v) / len(v) for k, v in agg.items()}
        if avg:
            avg["wait_any_frac"] = avg.get("SQ_WAIT_ANY", 0) / max(1.0, avg.get("SQ_WAVE_CYCLES", 1))
            avg["launches"] = len(agg.get("SQ_INSTS_VALU", []))
        print(json.dumps({"arm": arm, **{k: round(v, 4) if isinstance(v, float) else v for k, v in avg.items()}}))


if __name__ == "__main__":
    main()
