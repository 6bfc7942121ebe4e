#!/bin/bash
# Like tools/ab.sh, but keeps every bench line (launch counters included) in
# gpurun_out/ab_full_<workload>.jsonl and prints value, ms/frame, isolated
# kernel ms, wave rounds and traversal steps per variant.
# Usage: tools/ab_full.sh <workload> <rounds> a.so b.so,PT_SHADE_BATCH=24 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    IFS=, read -r lib envs <<< "$v"
    out=$(env PT_LIB="$lib" ${envs//,/ } timeout -k 10 120 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps 10 --warmup 2 2>/dev/null) || { echo "FAILED $v"; exit 3; }
    line=$(echo "$out" | tail -n 1)
    echo "{\"variant\": \"$v\", \"line\": $line}" >> "gpurun_out/ab_full_$WL.jsonl"
    echo "$v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; c=d["launch_counters"]; print(d["value"], d["ms_per_step"], r.get("isolated_kernel_ms"), c["wave_rounds"], c["wave_trav_steps"])')"
  done
done
