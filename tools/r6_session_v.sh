#!/bin/bash
# round 6, session v: render-stream placement arms, repeated (sessions s / u
# disagreed on the high-priority render streams): C3 shares N = 8 / 4 / 2 and
# the C4 N = 8 share, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
arms=("old:PT_XCHG_SIDE=1" "ns:" "pnd3:PT_BENCH_STREAM_PRIO=-1 PT_SMALL_DEPTH=3" "pn:PT_BENCH_STREAM_PRIO=-1"
      "rp:PT_RSTREAM_PRIO=-1" "cum:PT_RSTREAM_CUMASK=1" "cumd3:PT_RSTREAM_CUMASK=1 PT_SMALL_DEPTH=3")
for round in 1 2; do
  for cfg in "c3 8" "c3 4" "c3 2" "c4 8"; do
    set -- $cfg; wl=$1; n=$2
    for a in "${arms[@]}"; do
      name=${a%%:*}; envs=${a#*:}
      st=60; [ $wl = c4 ] && st=10
      out=$(env $envs timeout -k 10 150 python bench.py --workload $wl --no-cpu-baseline --no-extras --steps $st --warmup 3 \
            --emulate-shard $n --emulate-rank 0 2>/dev/null) || { echo "FAILED $name $wl $n"; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name $wl n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
    done
  done
done
