#!/bin/bash
# round 6, session t: render-slot streams at high priority + the exchange on
# the current stream (the new defaults) against the previous ones
# (PT_RSTREAM_PRIO=0 PT_XCHG_SIDE=1): GPU suite, C3 / C4 split emulation,
# whole C3 / C5 frames, the N = 2 rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6t_gpu_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r6t_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
arms=("new:" "old:PT_RSTREAM_PRIO=0 PT_XCHG_SIDE=1")
for round in 1 2; do
  for wl in c3 c4; do
    for n in 8 4 2; do
      [ $wl = c4 ] && [ $n != 8 ] && [ $round = 2 ] && continue
      for a in "${arms[@]}"; do
        name=${a%%:*}; envs=${a#*:}
        st=60; [ $wl = c4 ] && st=10
        out=$(env $envs timeout -k 10 150 python bench.py --workload $wl --no-cpu-baseline --no-extras --steps $st --warmup 3 \
              --emulate-shard $n --emulate-rank 0 2>/dev/null) || { echo "FAILED $name $wl $n"; exit 3; }
        echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name $wl n=$n', d['value'], d['ms_per_step'], d['exchange_ms'])"
      done
    done
  done
done
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 600 bash tools/ab.sh c3 3 $L "$L,PT_RSTREAM_PRIO=0" 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 bash tools/ab.sh c5 1 $L "$L,PT_RSTREAM_PRIO=0" 2>&1 | grep -v amdgpu.ids
REHEARSE_N=2 timeout -k 10 500 bash tools/rehearse_dist.sh
