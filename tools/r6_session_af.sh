#!/bin/bash
# round 6, session af: 8 vs 16 frames per launch (PT_MAX_FRAMES 16 build):
# C3 N = 8 / 4 shares (RCCL in the loop) and N = 1, 20 and 64 frames, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
  for k in 20 64; do
    for n in 8 4 1; do
      for f in 8 16; do
        em=""; [ $n -gt 1 ] && em="--emulate-shard $n --emulate-rank 0"
        out=$(PT_DIST_FORCE=1 timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps $k --warmup 3 \
              --frames-per-launch $f $em 2>gpurun_out/r6af_err.log) || { echo "FAILED n=$n f=$f"; tail -20 gpurun_out/r6af_err.log; exit 3; }
        echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('K=$k fpl=$f c3 n=$n', d['value'], d['ms_per_step'])"
      done
    done
  done
done
