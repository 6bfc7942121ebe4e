#!/bin/bash
# round 5: drained-queue detection with several heads (fix) vs HEAD (old):
# GPU suite on fix, then C5 / c5big (bands) and C3.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5aj_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5aj_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5aj_gpu_tests.log
timeout -k 10 900 bash tools/ab_suite.sh -H "old fix" -w "c5:2 c5big:1 c3:3" -o r5aj_fix _variants/fix.so _variants/old.so > /dev/null 2>&1 || { cat gpurun_out/r5aj_fix.txt; exit 1; }
cat gpurun_out/r5aj_fix.txt
