#!/bin/bash
# round 5: a launch with no frame in flight runs on the caller's stream
# (PT_IDLE_DIRECT): one-frame wall clock vs the cross-stream path and vs
# PT_PIPELINE=0; GPU suite on the new default.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5w_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5w_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5w_gpu_tests.log
timeout -k 10 600 bash tools/ab.sh c3 5 _variants/id1.so _variants/id0.so _variants/id0.so,PT_PIPELINE=0 > gpurun_out/r5w_ab_c3.txt 2>&1 || { cat gpurun_out/r5w_ab_c3.txt; exit 1; }
cat gpurun_out/r5w_ab_c3.txt
