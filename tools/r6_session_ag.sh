#!/bin/bash
# round 6, session ag: load balance of the strong split's deal -- every rank's
# share (one-GPU emulation, RCCL in the loop, 8 frames per launch, 40 frames)
# at N = 8 and N = 4 with the deal's tiles 32x32 (the FIFO) and 16x16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PT_DIST_FORCE=1
mkdir -p gpurun_out
for t in 32 16; do
  for n in 8 4; do
    for r in $(seq 0 $((n - 1))); do
      out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 40 --warmup 3 \
            --split-tile $t --emulate-shard $n --emulate-rank $r 2>gpurun_out/r6ag_err.log) || { echo "FAILED t=$t n=$n r=$r"; tail -20 gpurun_out/r6ag_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('tile=$t n=$n rank=$r', d['value'], d['ms_per_step'], d.get('exchange_ms'))"
    done
  done
done
