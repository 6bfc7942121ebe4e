#!/bin/bash
# A/B timing of library builds on the GPU box: alternates the variants ROUNDS
# times over one bench workload and prints each run's value (M samples/s),
# ms per frame (pipelined), the isolated kernel time, the resolve time and the
# wall-clock time of one frame alone (single_frame_ms).
# A variant is "lib.so" or "lib.so,VAR=val,VAR2=val" (environment for that arm).
# Usage: tools/ab.sh <workload> <rounds> a.so b.so,PT_SAMPLE_GROUP=2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=$1; R=$2; shift 2
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    IFS=, read -r lib envs <<< "$v"
    out=$(env PT_LIB="$lib" ${envs//,/ } timeout -k 10 120 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps 10 --warmup 2 2>/dev/null) || { echo "FAILED $v"; exit 3; }
    echo "$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], r.get("isolated_kernel_ms"), d["resolve_ms"], d["config"].get("single_frame_ms"))')"
  done
done
