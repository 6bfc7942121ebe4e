#!/bin/bash
# round 6, session ad: frames per launch 1 / 4 / 8 at the step counts a short
# driver run may use (20 and 40 timed frames, 3 warm-up), C3 shares N = 8 / 4 / 2
# with RCCL in the loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PT_DIST_FORCE=1
mkdir -p gpurun_out
for round in 1 2; do
  for k in 20 40; do
    for n in 8 4 2; do
      for f in 1 4 8; do
        out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps $k --warmup 3 \
              --frames-per-launch $f --emulate-shard $n --emulate-rank 0 2>gpurun_out/r6ad_err.log) || { echo "FAILED n=$n f=$f"; tail -20 gpurun_out/r6ad_err.log; exit 3; }
        echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('K=$k fpl=$f c3 n=$n', d['value'], d['ms_per_step'])"
      done
    done
  done
done
