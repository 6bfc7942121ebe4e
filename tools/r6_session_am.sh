#!/bin/bash
# round 6, session am: the library's Z-ordered launch (PT_TILE_ZORDER) --
# parity tests, then C5 / c5big / C4 / C3 default vs forced row-major (2 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread \
  -k "zorder or packed16 or frame_batch or render_tiles_device or pipelined" > gpurun_out/r6am_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r6am_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # label, bench args...
  local label=$1; shift
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras "$@" 2>gpurun_out/r6am_err.log) || { echo "FAILED $label"; tail -20 gpurun_out/r6am_err.log; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])"
}
for round in 1 2; do
  for wl in c5 c5big c4 c3; do
    case $wl in c3) st="--steps 64 --warmup 8";; c4) st="--steps 10 --warmup 3";; *) st="--steps 5 --warmup 2";; esac
    PT_TILE_ZORDER=0 run "$wl zorder=0" --workload $wl $st
    run "$wl zorder=default" --workload $wl $st
  done
done
