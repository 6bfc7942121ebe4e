#!/bin/bash
# round 6, session aj: the slowest ranks of the N = 8 C3 split per deal, 3
# rounds interleaved (RCCL in the loop, 8 frames per launch, 40 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PT_DIST_FORCE=1
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "diag 32 4" "diag 32 5" "diag3 32 0" "diag3 32 3" "diag3 16 1" "diag3 16 7" "diag5 16 7"; do
    set -- $cfg; deal=$1; t=$2; r=$3
    out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 40 --warmup 3 \
          --split-tile $t --split-deal $deal --emulate-shard 8 --emulate-rank $r 2>gpurun_out/r6aj_err.log) || { echo "FAILED"; tail -20 gpurun_out/r6aj_err.log; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3 deal=$deal tile=$t n=8 rank=$r', d['value'], d['ms_per_step'])"
  done
done
