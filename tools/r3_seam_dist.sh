set -e
mkdir -p gpurun_out
DAE=$(python3 -c "from dsgpuraytracing_amd import scenes; print(scenes.C1_DAE)")
timeout -k 10 240 ./dsgpuraytracing_amd/seam_bench "$DAE" 1024 1024 64 8 3 > gpurun_out/seam_native.json 2> gpurun_out/seam_native.err
cat gpurun_out/seam_native.json
PT_DIST_BACKEND=gloo PT_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2.log 2>&1
tail -c 3000 gpurun_out/dist2.log
