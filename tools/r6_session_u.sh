#!/bin/bash
# round 6, session u: why session t's default (render streams at the greatest
# priority from hipDeviceGetStreamPriorityRange) differs from session s's
# PT_RSTREAM_PRIO=-1 arm: arms + kernel traces of the C3 N = 8 share.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
python3 -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
arms=("new:" "m1:PT_RSTREAM_PRIO=-1" "m1ns:PT_RSTREAM_PRIO=-1 PT_XCHG_SIDE=0" "p0:PT_RSTREAM_PRIO=0" "old:PT_RSTREAM_PRIO=0 PT_XCHG_SIDE=1")
for round in 1 2; do
  for a in "${arms[@]}"; do
    name=${a%%:*}; envs=${a#*:}
    out=$(env $envs timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 3 \
          --emulate-shard 8 --emulate-rank 0 2>/dev/null) || { echo "FAILED $name"; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name c3 n=8', d['value'], d['ms_per_step'], d['exchange_ms'])"
  done
done
P="rocprofv3 --output-format csv --kernel-trace"
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 --emulate-shard 8 --emulate-rank 0"
timeout -k 10 240 $P -d gpurun_out/r6u/new -o new -- $B > gpurun_out/r6u_new.log 2>&1 && \
PT_RSTREAM_PRIO=-1 timeout -k 10 240 $P -d gpurun_out/r6u/m1 -o m1 -- $B > gpurun_out/r6u_m1.log 2>&1
