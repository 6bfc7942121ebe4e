#!/bin/bash
# round 6, session d: render-pipeline depth (PT_RENDER_SLOTS 2 = current, 3, 4, 8)
# on the one-GPU emulation of the C3 strong split (rank 0's share at N = 2 / 4 / 8)
# and on the whole C3 frame (tools/ab.sh, 2 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in dsgpuraytracing_amd/libptgpu.so _variants/slots3.so _variants/slots4.so _variants/slots8.so; do
  for n in 2 4 8; do
    out=$(PT_LIB=$v timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 20 --warmup 3 \
          --emulate-shard $n --emulate-rank 0 2>/dev/null) || { echo "FAILED $v $n"; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', $n, d['value'], d['ms_per_step'], d['exchange_ms'])"
  done
done
timeout -k 10 600 bash tools/ab.sh c3 2 dsgpuraytracing_amd/libptgpu.so _variants/slots3.so _variants/slots4.so _variants/slots8.so
