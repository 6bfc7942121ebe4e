#!/bin/bash
# round 6, session r: hardware-queue placement of the C3 split's streams.
# Session q's kernel trace showed render slots 0 and 2 on one HIP hardware
# queue (renders serialised) and the exchange's side stream on slot 1's.  Arms
# (one-GPU emulation, rank 0, N = 8 / 4 / 2, 2 rounds interleaved): stream
# priorities (HIP pools hardware queues per priority), the exchange on the
# current stream, small-launch depth 3, a third of the grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
python3 -c "import torch; s=torch.cuda.Stream(priority=-1); print('torch priority range', torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream,'priority_range') else None, 'stream prio', s.priority)"
arms=("base:" "prio:PT_BENCH_STREAM_PRIO=-1 PT_XCHG_PRIO=-1" "noside:PT_XCHG_SIDE=0" "depth3:PT_SMALL_DEPTH=3"
      "prio_d3:PT_BENCH_STREAM_PRIO=-1 PT_XCHG_PRIO=-1 PT_SMALL_DEPTH=3" "rprio:PT_RSTREAM_PRIO=-1" "div3:PT_SMALL_GRID_DIV=3")
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
P="rocprofv3 --output-format csv --kernel-trace"
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 --emulate-shard 8 --emulate-rank 0"
PT_BENCH_STREAM_PRIO=-1 PT_XCHG_PRIO=-1 timeout -k 10 240 $P -d gpurun_out/r6r/prio8 -o prio8 -- $B > gpurun_out/r6r_prio8.log 2>&1
