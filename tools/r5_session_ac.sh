#!/bin/bash
# round 5: 256-slot claims for frames launched while another is in flight
# (PT_CHUNK_BUSY): C3 5 rounds, framed C3 / C4 2 rounds; GPU suite first.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ac_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5ac_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5ac_gpu_tests.log
timeout -k 10 900 bash tools/ab.sh c3 5 _variants/busy1.so _variants/busy0.so > gpurun_out/r5ac_ab_c3.txt 2>&1 || { cat gpurun_out/r5ac_ab_c3.txt; exit 1; }
cat gpurun_out/r5ac_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c3f 2 _variants/busy1.so _variants/busy0.so > gpurun_out/r5ac_ab_c3f.txt 2>&1 || { cat gpurun_out/r5ac_ab_c3f.txt; exit 1; }
cat gpurun_out/r5ac_ab_c3f.txt
