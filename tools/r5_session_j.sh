#!/bin/bash
# round 5: step-selection simplification (PT_SEL_SIMPLE) and local waits for
# stack-spill loads (PT_SPILL_WAIT) A/B on C3 / C5; the 8-wide node (w8) on
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
# the compressed 4-wide node (nc = -DPT_NODE_COMPRESS=1): GPU suite on that library first
PT_LIB=_variants/nc.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5j_gpu_tests_nc.log 2>&1 || { echo "gpu tests (nc) failed"; tail -30 gpurun_out/r5j_gpu_tests_nc.log; exit 1; }
tail -2 gpurun_out/r5j_gpu_tests_nc.log
AB_FULL=1 timeout -k 10 500 bash tools/ab.sh c3 3 _variants/head.so _variants/sf.so _variants/sel0.so _variants/sw0.so _variants/nc.so > gpurun_out/r5j_ab_c3.txt 2>&1 || { cat gpurun_out/r5j_ab_c3.txt; exit 1; }
cat gpurun_out/r5j_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 2 _variants/head.so _variants/sf.so _variants/nc.so > gpurun_out/r5j_ab_c5.txt 2>&1 || { cat gpurun_out/r5j_ab_c5.txt; exit 1; }
cat gpurun_out/r5j_ab_c5.txt
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c4 1 _variants/head.so _variants/w8.so _variants/nc.so > gpurun_out/r5j_ab_c4.txt 2>&1 || { cat gpurun_out/r5j_ab_c4.txt; exit 1; }
cat gpurun_out/r5j_ab_c4.txt
