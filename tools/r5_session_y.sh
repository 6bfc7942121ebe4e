#!/bin/bash
# round 5: drain helpers (PT_HELPERS) and follow-up ray state by selects
# (PT_FOLLOW_SEL): GPU suite on the new default, then C3 / C5 A/Bs.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5y_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "PASS|FAIL" gpurun_out/r5y_gpu_tests.log | tail -5; tail -30 gpurun_out/r5y_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5y_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r5y_bench_c3.json 2>gpurun_out/r5y_bench_c3.err || { tail -20 gpurun_out/r5y_bench_c3.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5y_bench_c3.json').read().strip().splitlines()[-1]); c=d['config']
print('value', d['value'], 'single', c.get('single_frame_ms'), 'api', c.get('single_frame_api_ms'), 'sync', c.get('sync_floor_ms'), 'iso', d['roofline'].get('isolated_kernel_ms'))"
timeout -k 10 900 bash tools/ab.sh c3 5 _variants/c_hp.so _variants/c_hp.so,PT_NO_HELPERS=1 _variants/b_fs.so _variants/a_base.so > gpurun_out/r5y_ab_c3.txt 2>&1 || { cat gpurun_out/r5y_ab_c3.txt; exit 1; }
cat gpurun_out/r5y_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c5 2 _variants/c_hp.so _variants/a_base.so > gpurun_out/r5y_ab_c5.txt 2>&1 || { cat gpurun_out/r5y_ab_c5.txt; exit 1; }
cat gpurun_out/r5y_ab_c5.txt
