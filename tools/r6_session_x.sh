#!/bin/bash
# round 6, session x: render streams created at context creation (PT_EAGER_SLOTS)
# x small-launch depth (PT_SMALL_DEPTH), with and without RCCL in the loop
# (PT_DIST_FORCE=1): C3 shares N = 8 / 4 / 2, whole C3 (tools/ab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
arms=("base:" "e3d3:PT_EAGER_SLOTS=3 PT_SMALL_DEPTH=3" "e4:PT_EAGER_SLOTS=4" "e3:PT_EAGER_SLOTS=3" "d3:PT_SMALL_DEPTH=3")
for f in 0 1; do
  for round in 1 2; do
    for n in 8 4 2; do
      for a in "${arms[@]}"; do
        name=${a%%:*}; envs=${a#*:}
        out=$(env PT_DIST_FORCE=$f $envs timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 3 \
              --emulate-shard $n --emulate-rank 0 2>gpurun_out/r6x_err.log) || { echo "FAILED $name $n"; tail -20 gpurun_out/r6x_err.log; exit 3; }
        echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('force=$f $name c3 n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
      done
    done
  done
done
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 600 bash tools/ab.sh c3 2 $L "$L,PT_EAGER_SLOTS=3" "$L,PT_EAGER_SLOTS=4" 2>&1 | grep -v amdgpu.ids
