#!/bin/bash
# One rocprofv3 --pmc pass per arm over `bench.py --workload <wl>` with
# PT_PIPELINE=0 (every launch alone), then the render kernel's per-launch mean
# of each counter per arm.  Counters must fit one pass (MI355X_MICROARCH.md:
# <= 8 SQ, <= 4 TCC, ...).  An arm is "name=lib.so[,VAR=v...]".
# Usage: tools/pmc_pass.sh <workload> "TCC_HIT_sum TCC_MISS_sum" w4=_variants/w4.so w8=_variants/w8.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=$1; CTRS=$2; shift 2
OUT=gpurun_out/pmcpass_${WL}_$(echo "$CTRS" | tr ' ' '_' | cut -c1-40)
rm -rf "$OUT"
for arm in "$@"; do
  name=${arm%%=*}; rest=${arm#*=}
  IFS=, read -r lib envs <<< "$rest"
  env PT_PIPELINE=0 PT_LIB="$lib" ${envs//,/ } timeout -s KILL 120 rocprofv3 --output-format csv \
    --pmc $CTRS -d "$OUT/$name" -o p -- python3 bench.py --workload "$WL" --steps 3 --warmup 1 \
    --no-cpu-baseline --no-extras > /dev/null 2>&1 || { echo "FAILED $name"; exit 3; }
done
python3 - "$OUT" "$WL" <<'PY'
import csv, glob, json, os, sys, collections
out, wl = sys.argv[1:]
for arm in sorted(os.listdir(out)):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{arm}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "render_kernel<false" in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in per.items():
            vals[c].append(v)
    print(json.dumps({"arm": arm, "workload": wl, **{c: round(sum(v) / len(v), 1) for c, v in sorted(vals.items())},
                      "launches": max((len(v) for v in vals.values()), default=0)}))
PY
