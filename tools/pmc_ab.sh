#!/bin/bash
# HBM counters of library variants on one workload (PT_PIPELINE=0: every
# render alone), one counter per rocprofv3 pass; writes
# gpurun_out/pmcab/<workload>_<variant>_<counter>/ and prints, per variant,
# the render kernel's mean FETCH_SIZE / WRITE_SIZE per launch (KB).
# Usage: tools/pmc_ab.sh <workload> <variant.so> ...
#   (PMC_PASSES="WRITE_SIZE FETCH_SIZE TCC_HIT_sum,TCC_MISS_sum": other passes; a comma joins
#   counters into one pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=$1; shift
for lib in "$@"; do
  v=$(basename "$lib" .so)
  for c in ${PMC_PASSES:-WRITE_SIZE FETCH_SIZE}; do
    PT_PIPELINE=0 PT_LIB=$lib timeout -s KILL 120 rocprofv3 --output-format csv --pmc ${c//,/ } -d gpurun_out/pmcab/${WL}_${v}_$c -o p -- python3 bench.py --workload "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
    python3 - "$WL" "$v" "$c" <<'PY'
import csv, glob, sys
wl, v, c = sys.argv[1:]
vals = {}
for f in glob.glob(f"gpurun_out/pmcab/{wl}_{v}_{c}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "render_kernel<false" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for name, x in sorted(vals.items()):
    print(wl, v, name, round(sum(x) / max(1, len(x)), 1), "(KB for *_SIZE) per launch over", len(x))
PY
  done
done
