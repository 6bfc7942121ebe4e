#!/bin/bash
# round 5: the resolve on the render stream (PT_RESOLVE_ON_RS) on top of the
# queue-head reset: one-frame wall clock; GPU suite on the new default.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5v_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5v_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5v_gpu_tests.log
timeout -k 10 600 bash tools/ab.sh c3 5 _variants/new2.so _variants/rs0.so _variants/rr0.so > gpurun_out/r5v_ab_c3.txt 2>&1 || { cat gpurun_out/r5v_ab_c3.txt; exit 1; }
cat gpurun_out/r5v_ab_c3.txt
