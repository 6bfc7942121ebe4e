#!/bin/bash
# round 6, session al: the tile order on the large frames (C5, C4; 3 rounds
# interleaved), and the N = 4 C3 split's deals (diag3 vs diag, 32x32 tiles),
# every rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label, bench args...
  local label=$1; shift
  out=$(timeout -k 10 150 python bench.py --no-cpu-baseline --no-extras "$@" 2>gpurun_out/r6al_err.log) || { echo "FAILED $label"; tail -20 gpurun_out/r6al_err.log; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])"
}
for round in 1 2 3; do
  for cfg in "c5 32 rows" "c5 16 morton" "c5 32 morton" "c4 32 rows" "c4 32 morton"; do
    set -- $cfg
    run "$1 n=1 tile=$2 order=$3" --workload $1 --steps 8 --warmup 2 --tile $2 --tile-order $3
  done
done
export PT_DIST_FORCE=1
for deal in diag3 diag; do
  for r in 0 1 2 3; do
    run "c3 deal=$deal tile=32 n=4 rank=$r" --workload c3 --steps 40 --warmup 3 --split-deal $deal --emulate-shard 4 --emulate-rank $r
  done
done
