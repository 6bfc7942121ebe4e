#!/bin/bash
# round 6, session p: hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP's
# default vs 8) for the whole C3 frame (tools/ab.sh, 3 rounds) and the C3 split
# emulation (rank 0 at N = 2 / 4 / 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 800 bash tools/ab.sh c3 3 $L $L,GPU_MAX_HW_QUEUES=8 > gpurun_out/r6p_ab_hwq.txt 2>&1 || { cat gpurun_out/r6p_ab_hwq.txt; exit 1; }
cat gpurun_out/r6p_ab_hwq.txt
for q in 4 8; do
  for n in 2 4 8; do
    out=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 30 --warmup 3 \
          --emulate-shard $n --emulate-rank 0 2>/dev/null) || { echo "FAILED $q $n"; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('hwq=$q n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
  done
done
