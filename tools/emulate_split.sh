#!/bin/bash
# One-GPU emulation of the multi-GPU C4 split: times rank r's share of an
# N-way diagonal tile deal (bench.py --emulate-shard N --emulate-rank r).
# Usage: tools/emulate_split.sh [workload] -> "N rank value ms_per_step" lines
# (PT_DIST_FORCE=1 in the environment: the exchange goes through a one-rank
# RCCL group and torch's collective stream, as on a rank of an N-GPU run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
WL=${1:-c4}
for n in 1 2 4 8; do
  for r in 0 $((n > 1 ? n - 1 : 0)); do
    out=$(timeout -k 10 120 python bench.py --workload "$WL" --no-cpu-baseline --no-extras --steps "${EMU_STEPS:-40}" \
          --emulate-shard "$n" --emulate-rank "$r" 2>/dev/null) || { echo "FAILED $n $r"; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print($n, $r, d['value'], d['ms_per_step'])"
  done
done
