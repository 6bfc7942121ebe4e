#!/bin/bash
# round 6, session e: the C3 strong-split share (one-GPU emulation, rank 0) with a
# smaller resident grid per launch (PT_WAVES_PER_CU) and more frames in flight
# (PT_RENDER_SLOTS variants): more work slots per lane per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
run() {  # lib n wpc
  out=$(PT_LIB=$1 PT_WAVES_PER_CU=$3 timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 30 --warmup 3 \
        --emulate-shard $2 --emulate-rank 0 2>/dev/null) || { echo "FAILED $*"; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 n=$2 wpc=$3', d['value'], d['ms_per_step'])"
}
L=dsgpuraytracing_amd/libptgpu.so
for n in 8 4 2; do
  run $L $n 20
  run $L $n 10
  run _variants/slots4.so $n 10
  run _variants/slots4.so $n 5
  run _variants/slots8.so $n 5
  run _variants/slots8.so $n 3
done
run $L 1 20
run _variants/slots4.so 1 10
