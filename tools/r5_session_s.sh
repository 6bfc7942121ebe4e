#!/bin/bash
# round 5: SAH-optimal (DP) BVH4 collapse (default now) vs the greedy collapse
# (PT_COLLAPSE=area), GPU tree and host SAH tree; GPU suite on the default.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_*.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5s_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5s_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5s_gpu_tests.log
L=_variants/dp.so
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c3 3 $L $L,PT_COLLAPSE=area > gpurun_out/r5s_ab_c3.txt 2>&1 || { cat gpurun_out/r5s_ab_c3.txt; exit 1; }
cat gpurun_out/r5s_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c3 1 $L,PT_BVH_BUILD=sah $L,PT_BVH_BUILD=sah,PT_COLLAPSE=area > gpurun_out/r5s_ab_c3sah.txt 2>&1 || { cat gpurun_out/r5s_ab_c3sah.txt; exit 1; }
cat gpurun_out/r5s_ab_c3sah.txt
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c5 2 $L $L,PT_COLLAPSE=area > gpurun_out/r5s_ab_c5.txt 2>&1 || { cat gpurun_out/r5s_ab_c5.txt; exit 1; }
cat gpurun_out/r5s_ab_c5.txt
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c4 1 $L $L,PT_COLLAPSE=area > gpurun_out/r5s_ab_c4.txt 2>&1 || { cat gpurun_out/r5s_ab_c4.txt; exit 1; }
cat gpurun_out/r5s_ab_c4.txt
timeout -k 10 300 bash tools/ab.sh c5big 1 $L $L,PT_COLLAPSE=area > gpurun_out/r5s_ab_c5big.txt 2>&1 || { cat gpurun_out/r5s_ab_c5big.txt; exit 1; }
cat gpurun_out/r5s_ab_c5big.txt
