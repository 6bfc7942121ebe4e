#!/bin/bash
# round 5: the resolve zeroes its launch's queue heads (PT_RESOLVE_RESETS), so a
# launch needs no memset in front of the render -- GPU suite, A/B (one-frame
# wall clock is the column that should move).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5u_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5u_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5u_gpu_tests.log
timeout -k 10 500 bash tools/ab.sh c3 4 _variants/new.so _variants/rr0.so > gpurun_out/r5u_ab_c3.txt 2>&1 || { cat gpurun_out/r5u_ab_c3.txt; exit 1; }
cat gpurun_out/r5u_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c4 1 _variants/new.so _variants/rr0.so > gpurun_out/r5u_ab_c4.txt 2>&1 || { cat gpurun_out/r5u_ab_c4.txt; exit 1; }
cat gpurun_out/r5u_ab_c4.txt
