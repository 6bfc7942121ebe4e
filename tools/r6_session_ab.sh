#!/bin/bash
# round 6, session ab: frame batches up to 8 frames per launch: tests, then the
# C3 shares / whole frame at 4 and 8 frames per launch (RCCL in the loop, 64
# frames), and C4 / C5 single-GPU lines at 1 / 4 frames per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -k "frame_batch" -x -v --timeout 120 --timeout-method thread > gpurun_out/r6ab_tests.log 2>&1
rc=$?; tail -n 6 gpurun_out/r6ab_tests.log; [ $rc -eq 0 ] || exit $rc
export PT_DIST_FORCE=1
for round in 1 2; do
  for n in 8 4 2 1; do
    for f in 1 4 8; do
      em=""; [ $n -gt 1 ] && em="--emulate-shard $n --emulate-rank 0"
      out=$(timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --no-extras --steps 64 --warmup 8 \
            --frames-per-launch $f $em 2>gpurun_out/r6ab_err.log) || { echo "FAILED n=$n f=$f"; tail -20 gpurun_out/r6ab_err.log; exit 3; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fpl=$f c3 n=$n', d['value'], d['ms_per_step'], d.get('exchange_ms'))"
    done
  done
done
for wl in c4 c5; do
  for f in 1 4; do
    st=8; [ $wl = c5 ] && st=4
    out=$(timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-extras --steps $st --warmup 2 \
          --frames-per-launch $f 2>gpurun_out/r6ab_err.log) || { echo "FAILED $wl f=$f"; tail -20 gpurun_out/r6ab_err.log; exit 3; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fpl=$f $wl n=1', d['value'], d['ms_per_step'])"
  done
done
