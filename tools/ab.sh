#!/bin/bash
# A/B timing of library builds on the GPU box: alternates the variants ROUNDS
# times over one bench workload and prints, per run: value (M samples/s), ms
# per frame (pipelined), the isolated kernel time, the resolve time and the
# wall-clock time of one frame alone (single_frame_ms); with AB_FULL=1 also
# the launch's shading rounds and wave traversal steps (each line is kept in
# gpurun_out/ab_full_<workload>.jsonl).
# A variant is "lib.so" or "lib.so,VAR=val,VAR2=val" (environment for that arm).
# Usage: tools/ab.sh <workload> <rounds> a.so b.so,PT_SAMPLE_GROUP=2 ...
#   (tools/ab_suite.sh runs the GPU suite, image hashes and several workloads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    IFS=, read -r lib envs <<< "$v"
    out=$(env PT_LIB="$lib" ${envs//,/ } timeout -k 10 300 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps 10 --warmup 2 2>/dev/null) || { echo "FAILED $v"; exit 3; }
    line=$(echo "$out" | tail -n 1)
    [ -n "$AB_FULL" ] && echo "{\"variant\": \"$v\", \"line\": $line}" >> "gpurun_out/ab_full_$WL.jsonl"
    echo "$v $(echo "$line" | AB_FULL="$AB_FULL" python -c '
import json, os, sys
d = json.loads(sys.stdin.read()); r = d["roofline"]; c = d["launch_counters"]
x = [d["value"], d["ms_per_step"], r.get("isolated_kernel_ms"), d["resolve_ms"], d["config"].get("single_frame_ms")]
if os.environ.get("AB_FULL"):
    x += [c["wave_rounds"], c["wave_trav_steps"]]
print(*x)')"
  done
done
