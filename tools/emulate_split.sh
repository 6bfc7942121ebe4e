#!/bin/bash
# One-GPU emulation of the multi-GPU strong split: times EVERY rank's share of
# the N-way tile deal (bench.py --emulate-shard N --emulate-rank r; the deal is
# bench.py's default, --split-deal auto), then per N the slowest rank -- the
# N-GPU frame time -- and the efficiency t(1) / (N * slowest).
# Usage: tools/emulate_split.sh [workload] -> "N rank value ms_per_step" lines
# and "N slowest <ms> eff <frac>" lines
# (PT_DIST_FORCE=1 in the environment: the exchange goes through a one-rank
# RCCL group and torch's collective stream, as on a rank of an N-GPU run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=${1:-c4}
t1=""
for n in 1 2 4 8; do
  slow=0
  for r in $(seq 0 $((n - 1))); do
    out=$(timeout -k 10 120 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps "${EMU_STEPS:-40}" \
          --emulate-shard "$n" --emulate-rank "$r" 2>/dev/null) || { echo "FAILED $n $r"; exit 3; }
    ms=$(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])")
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print($n, $r, d['value'], d['ms_per_step'])"
    slow=$(python -c "print(max($slow, $ms))")
  done
  [ -n "$t1" ] || t1=$slow
  python -c "print($n, 'slowest', $slow, 'eff', round($t1 / ($n * $slow), 3))"
done
