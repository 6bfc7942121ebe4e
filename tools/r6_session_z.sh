#!/bin/bash
# round 6, session z: grid fraction of the small launches (PT_WAVES_PER_CU
# 10 = the default half grid, 12, 15, 20) for the C3 shares, RCCL in the loop
# (PT_DIST_FORCE=1: render slots on two hardware queues, see session y).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PT_DIST_FORCE=1
mkdir -p gpurun_out
for round in 1 2; do
  for n in 8 4 2; do
    for w in def 12 15 20; do
      envs=""; [ $w != def ] && envs="PT_WAVES_PER_CU=$w"
      out=$(env $envs timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 3 \
            --emulate-shard $n --emulate-rank 0 2>gpurun_out/r6z_err.log) || { echo "FAILED $w $n"; tail -20 gpurun_out/r6z_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('wpc=$w c3 n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
    done
  done
done
