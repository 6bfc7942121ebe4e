#!/bin/bash
# round 5: queue bands for large frames (P.qbands auto) vs interleaved
# (PT_QUEUE_BANDS=0): C4 2 rounds, C5 / c5big 1, C3 2; GPU suite first.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ae_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5ae_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5ae_gpu_tests.log
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 900 bash tools/ab_suite.sh -w "c4:2 c5:1 c5big:1 c3:2" -o r5ae_bands_auto $L $L,PT_QUEUE_BANDS=0 > /dev/null 2>&1 || { cat gpurun_out/r5ae_bands_auto.txt; exit 1; }
cat gpurun_out/r5ae_bands_auto.txt
