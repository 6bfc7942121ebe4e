#!/bin/bash
# round 6, session aa: frame batches (pt_render_frames_device, the MF kernel):
# bit-identity tests, then the C3 split's shares and the whole frame at
# 1 / 2 / 4 frames per launch (one-GPU emulation, RCCL in the loop, 60 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -k "frame_batch" tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6aa_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/r6aa_tests.log; [ $rc -eq 0 ] || exit $rc
export PT_DIST_FORCE=1
for round in 1 2; do
  for n in 8 4 2 1; do
    for f in 1 2 4; do
      em=""; [ $n -gt 1 ] && em="--emulate-shard $n --emulate-rank 0"
      out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 4 \
            --frames-per-launch $f $em 2>gpurun_out/r6aa_err.log) || { echo "FAILED n=$n f=$f"; tail -20 gpurun_out/r6aa_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fpl=$f c3 n=$n', d['value'], d['ms_per_step'], d.get('exchange_ms'))"
    done
  done
done
