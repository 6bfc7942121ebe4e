#!/bin/bash
# round 6, session ah: every rank's share of the N = 8 C3 split for several
# tile deals (diagK: (column + K * row) mod N) and tile sizes -- the slowest
# rank sets the frame (RCCL in the loop, 8 frames per launch, 40 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PT_DIST_FORCE=1
mkdir -p gpurun_out
for cfg in "diag 32" "diag3 32" "diag5 32" "diag3 16" "diag5 16"; do
  set -- $cfg; deal=$1; t=$2
  for r in 0 1 2 3 4 5 6 7; do
    out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 40 --warmup 3 \
          --split-tile $t --split-deal $deal --emulate-shard 8 --emulate-rank $r 2>gpurun_out/r6ah_err.log) || { echo "FAILED $deal $t $r"; tail -20 gpurun_out/r6ah_err.log; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('deal=$deal tile=$t n=8 rank=$r', d['value'], d['ms_per_step'])"
  done
done
