#!/bin/bash
# N-rank bench flow rehearsed on ONE GPU: every rank on cuda:0, gloo (host-staged exchange).
# Default N > 1 line: the C3 frame split over the ranks with the pipelined gather
# (efficiency is null here: the ranks share one device); companions c4_strong and c3_weak.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for n in ${REHEARSE_N:-2 4}; do
  PT_DIST_BACKEND=gloo PT_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/rehearse_$n.log 2>&1 || { tail -30 gpurun_out/rehearse_$n.log; exit 1; }
  tail -n 1 gpurun_out/rehearse_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print($n, d['value'], d['ms_per_step'], d['scaling'], d['config']['parallelism'], 'single_gpu_value', d.get('single_gpu_value'),
      'efficiency', d.get('efficiency'), 'shared_device', d.get('shared_device'), 'exchange_ms', d.get('exchange_ms'),
      'traced', d.get('traced_samples_per_s_M'), 'per_rank', d.get('per_rank'))
for k, v in (d.get('companions') or {}).items():
    print('  ', k, {x: v.get(x) for x in ('value', 'ms_per_frame', 'single_gpu_value', 'efficiency', 'shared_device', 'kernel_ms_slowest_over_mean', 'reduce_ms')})"
done
