#!/bin/bash
# round 5: follow-up ray state by selects (PT_FOLLOW_SEL) A/B on C3 and C5;
# the host-side share of one frame's wall clock (bench single_frame_api_ms);
# GPU suite on the new default.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5x_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5x_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5x_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r5x_bench_c3.json 2>gpurun_out/r5x_bench_c3.err || { tail -20 gpurun_out/r5x_bench_c3.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5x_bench_c3.json').read().strip().splitlines()[-1]); c=d['config']
print('value', d['value'], 'single', c.get('single_frame_ms'), 'api', c.get('single_frame_api_ms'), 'sync', c.get('sync_floor_ms'))"
timeout -k 10 600 bash tools/ab.sh c3 5 _variants/fs1.so _variants/fs0.so > gpurun_out/r5x_ab_c3.txt 2>&1 || { cat gpurun_out/r5x_ab_c3.txt; exit 1; }
cat gpurun_out/r5x_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c5 2 _variants/fs1.so _variants/fs0.so > gpurun_out/r5x_ab_c5.txt 2>&1 || { cat gpurun_out/r5x_ab_c5.txt; exit 1; }
cat gpurun_out/r5x_ab_c5.txt
