#!/bin/bash
# round 6, session an: does the library's Z-order take (probe), and C5's
# bench-side Z-order vs the library's, arms in rotated order (2 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/zorder_probe.py c5 || exit 3
run() {  # label, bench args...
  local label=$1; shift
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras "$@" 2>gpurun_out/r6an_err.log) || { echo "FAILED $label"; tail -20 gpurun_out/r6an_err.log; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])"
}
for round in 1 2; do
  run "c5 bench-morton lib-default" --workload c5 --steps 5 --warmup 2 --tile-order morton
  PT_TILE_ZORDER=0 run "c5 bench-morton lib-zorder=0" --workload c5 --steps 5 --warmup 2 --tile-order morton
  run "c5 bench-rows lib-default" --workload c5 --steps 5 --warmup 2
  PT_TILE_ZORDER=0 run "c5 bench-rows lib-zorder=0" --workload c5 --steps 5 --warmup 2
done
