# N-rank bench flow rehearsed on ONE GPU: every rank on cuda:0, gloo (host-staged exchange).
set -e
mkdir -p gpurun_out
for n in 2 4; do
  PT_DIST_BACKEND=gloo PT_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/rehearse_$n.log 2>&1
  tail -n 1 gpurun_out/rehearse_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'], d['scaling'], d['config']['parallelism'], d['config']['spp_total'], d['dist'], d.get('per_rank'), {k: (v['value'], v['ms_per_frame'], v.get('single_gpu_value'), v.get('efficiency'), v.get('kernel_ms_slowest_over_mean'), v.get('per_rank')) for k, v in (d.get('companions') or {}).items()})"
done
PT_DIST_BACKEND=gloo PT_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29610 bench.py --gpus 2 --steps 3 --warmup 1 --workload c4 --scaling strong > gpurun_out/rehearse_c4.log 2>&1
tail -n 1 gpurun_out/rehearse_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 strong', d['value'], d['ms_per_step'], d['scaling'], d['config']['parallelism'], d.get('per_rank'))"
