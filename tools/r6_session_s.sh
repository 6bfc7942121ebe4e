#!/bin/bash
# round 6, session s: follow-up of session r (profiles/r6/ab_stream_queues.txt).
# Four active hardware queues at most: render slots on three distinct queues
# and the resolve + exchange on one (PT_XCHG_SIDE=0), by stream priority.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
arms=("base:" "prio_d3:PT_BENCH_STREAM_PRIO=-1 PT_XCHG_PRIO=-1 PT_SMALL_DEPTH=3"
      "prio_ns_d3:PT_BENCH_STREAM_PRIO=-1 PT_XCHG_SIDE=0 PT_SMALL_DEPTH=3"
      "prio_ns:PT_BENCH_STREAM_PRIO=-1 PT_XCHG_SIDE=0"
      "rprio_d3:PT_RSTREAM_PRIO=-1 PT_SMALL_DEPTH=3"
      "rprio_ns_d3:PT_RSTREAM_PRIO=-1 PT_XCHG_SIDE=0 PT_SMALL_DEPTH=3"
      "rprio_ns:PT_RSTREAM_PRIO=-1 PT_XCHG_SIDE=0")
for round in 1 2; do
  for n in 8 4 2; do
    for a in "${arms[@]}"; do
      name=${a%%:*}; envs=${a#*:}
      out=$(env $envs timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 \
            --emulate-shard $n --emulate-rank 0 2>/dev/null) || { echo "FAILED $name $n"; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
    done
  done
done
# the whole C3 frame (large launches, 2 slots) under the two priority schemes
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 600 bash tools/ab.sh c3 2 $L "$L,PT_BENCH_STREAM_PRIO=-1,PT_XCHG_SIDE=0" "$L,PT_RSTREAM_PRIO=-1" 2>&1 | grep -v amdgpu.ids
P="rocprofv3 --output-format csv --kernel-trace"
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 --emulate-shard 4 --emulate-rank 0"
PT_BENCH_STREAM_PRIO=-1 PT_XCHG_SIDE=0 PT_SMALL_DEPTH=3 timeout -k 10 240 $P -d gpurun_out/r6s/pnd3 -o pnd3 -- $B > gpurun_out/r6s_pnd3.log 2>&1
PT_RSTREAM_PRIO=-1 PT_XCHG_SIDE=0 PT_SMALL_DEPTH=3 timeout -k 10 240 $P -d gpurun_out/r6s/rnd3 -o rnd3 -- $B > gpurun_out/r6s_rnd3.log 2>&1
