#!/bin/bash
# A/B timing of library builds on the GPU box: alternates the variants ROUNDS
# times over one bench workload and prints each run's value and kernel time.
# A variant is "lib.so" or "lib.so,VAR=val,VAR2=val" (environment for that arm).
# Usage: tools/ab.sh <workload> <rounds> a.so b.so,PT_BVH_ORDER=bfs ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=$1; R=$2; shift 2
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    IFS=, read -r lib envs <<< "$v"
    out=$(env PT_LIB="$lib" ${envs//,/ } timeout -k 10 120 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps 10 --warmup 2 2>/dev/null) || { echo "FAILED $v"; exit 3; }
    echo "$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["roofline"]["kernel_ms"], d["resolve_ms"])')"
  done
done
