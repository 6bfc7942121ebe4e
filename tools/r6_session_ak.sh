#!/bin/bash
# round 6, session ak: the tile FIFO's edge and order at N = 1 (C3, 8 frames
# per launch), 2 rounds interleaved; then the N = 8 split of 16x16 tiles dealt
# by 32x32 blocks (diag3), every rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label, bench args...
  local label=$1; shift
  out=$(timeout -k 10 150 python bench.py --no-cpu-baseline --no-extras "$@" 2>gpurun_out/r6ak_err.log) || { echo "FAILED $label"; tail -20 gpurun_out/r6ak_err.log; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])"
}
for round in 1 2; do
  for cfg in "32 rows" "16 rows" "8 rows" "32 morton" "16 morton" "8 morton"; do
    set -- $cfg
    run "c3 n=1 tile=$1 order=$2" --workload c3 --steps 64 --warmup 8 --tile $1 --tile-order $2
  done
done
for cfg in "c4 32 rows" "c4 16 rows" "c4 16 morton" "c5 32 rows" "c5 16 rows" "c5 16 morton"; do
  set -- $cfg
  run "$1 n=1 tile=$2 order=$3" --workload $1 --steps 8 --warmup 2 --tile $2 --tile-order $3
done
export PT_DIST_FORCE=1
for r in 0 1 2 3 4 5 6 7; do
  run "c3 deal=diag3 tile=16 block=32 n=8 rank=$r" --workload c3 --steps 40 --warmup 3 --split-tile 16 --deal-block 32 \
      --split-deal diag3 --emulate-shard 8 --emulate-rank $r
done
