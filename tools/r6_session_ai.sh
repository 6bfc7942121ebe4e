#!/bin/bash
# round 6, session ai: PT_FLAG_PACKED16 tests, then every rank's share of the
# C3 split at N = 8 / 4 / 2 with the deal of 16x16 tiles (diag3) against the
# 32x32 diagonal deal, and C4 at N = 8 (RCCL in the loop, 40 / 10 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -k "packed or frame_batch" tests/test_gpu_rccl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ai_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r6ai_tests.log; [ $rc -eq 0 ] || exit $rc
export PT_DIST_FORCE=1
for cfg in "diag3 16" "diag 32"; do
  set -- $cfg; deal=$1; t=$2
  for n in 8 4 2; do
    for r in $(seq 0 $((n - 1))); do
      out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 40 --warmup 3 \
            --split-tile $t --split-deal $deal --emulate-shard $n --emulate-rank $r 2>gpurun_out/r6ai_err.log) || { echo "FAILED"; tail -20 gpurun_out/r6ai_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3 deal=$deal tile=$t n=$n rank=$r', d['value'], d['ms_per_step'], d.get('exchange_ms'))"
    done
  done
  for r in 0 1 2 3 4 5 6 7; do
    out=$(timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --no-extras --steps 10 --warmup 2 \
          --split-tile $t --split-deal $deal --emulate-shard 8 --emulate-rank $r 2>gpurun_out/r6ai_err.log) || { echo "FAILED"; tail -20 gpurun_out/r6ai_err.log; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c4 deal=$deal tile=$t n=8 rank=$r', d['value'], d['ms_per_step'], d.get('exchange_ms'))"
  done
done
