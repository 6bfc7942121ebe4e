#!/bin/bash
# round 6, session f: the C3 strong-split share (one-GPU emulation, rank 0): claim
# size (PT_CHUNK_SLOTS 64 vs 128) x resident grid x pipeline depth; pipelined
# ms per frame, the lone launch (HIP events) and one frame alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
run() {  # lib n wpc chunk
  out=$(PT_LIB=$1 PT_WAVES_PER_CU=$3 PT_CHUNK_SLOTS=$4 timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 30 --warmup 3 \
        --emulate-shard $2 --emulate-rank 0 2>/dev/null) || { echo "FAILED $*"; exit 3; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 n=$2 wpc=$3 chunk=$4', d['value'], d['ms_per_step'], 'lone', d['roofline']['isolated_kernel_ms'], 'single', d['config']['single_frame_ms'], 'group', d['launch']['group_spp'])"
}
L=dsgpuraytracing_amd/libptgpu.so
S=_variants/slots4.so
for n in 8 4 2; do
  run $L $n 20 128
  run $L $n 20 64
  run $S $n 10 128
  run $S $n 10 64
  run $S $n 20 64
done
