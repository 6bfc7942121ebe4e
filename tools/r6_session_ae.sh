#!/bin/bash
# round 6, session ae: the N = 1 headline at 1 / 4 / 8 frames per launch with
# the default step counts (20 timed, 3 warm-up) and at 64 frames, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2 3; do
  for k in 20 64; do
    for f in 1 4 8; do
      out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps $k --warmup 3 \
            --frames-per-launch $f 2>gpurun_out/r6ae_err.log) || { echo "FAILED k=$k f=$f"; tail -20 gpurun_out/r6ae_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('K=$k fpl=$f c3 n=1', d['value'], d['ms_per_step'])"
    done
  done
done
