#!/bin/bash
# round 6, session w: the C3 / C4 split shares with the exchange through RCCL
# and torch's collective stream (a one-rank "nccl" group, PT_DIST_FORCE=1), as
# on every rank of an N-GPU run: stream-placement arms, 2 rounds; kernel trace
# of the pnd3 arm.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
export PT_DIST_FORCE=1
arms=("ns:" "nsd3:PT_SMALL_DEPTH=3" "pnd3:PT_BENCH_STREAM_PRIO=-1 PT_SMALL_DEPTH=3"
      "pnd3h:PT_BENCH_STREAM_PRIO=-1 PT_SMALL_DEPTH=3 PT_NCCL_HIPRIO=1" "pn:PT_BENCH_STREAM_PRIO=-1" "old:PT_XCHG_SIDE=1")
for round in 1 2; do
  for cfg in "c3 8" "c3 4" "c4 8"; do
    set -- $cfg; wl=$1; n=$2
    for a in "${arms[@]}"; do
      name=${a%%:*}; envs=${a#*:}
      st=60; [ $wl = c4 ] && st=10
      out=$(env $envs timeout -k 10 150 python bench.py --workload $wl --no-cpu-baseline --no-extras --steps $st --warmup 3 \
            --emulate-shard $n --emulate-rank 0 2>gpurun_out/r6w_err.log) || { echo "FAILED $name $wl $n"; tail -20 gpurun_out/r6w_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name $wl n=$n', d['value'], d['ms_per_step'], d['exchange_ms'], d['dist']['world_size'])"
    done
  done
done
P="rocprofv3 --output-format csv --kernel-trace"
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 --emulate-shard 8 --emulate-rank 0"
PT_BENCH_STREAM_PRIO=-1 PT_SMALL_DEPTH=3 timeout -k 10 240 $P -d gpurun_out/r6w/pnd3 -o pnd3 -- $B > gpurun_out/r6w_pnd3.log 2>&1
