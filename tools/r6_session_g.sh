#!/bin/bash
# round 6, session g: the small-launch shape.  C3 strong-split emulation
# (rank 0 and rank N-1 at N = 2 / 4 / 8) and C4 (unaffected: large shares),
# the whole C3 frame with the shape on / off (tools/ab.sh, 3 rounds), the new
# bit-identity test and the full-size tests, the node-step census, a bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_rccl.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r6g_tests.log 2>&1 || { tail -40 gpurun_out/r6g_tests.log; exit 1; }
tail -2 gpurun_out/r6g_tests.log
timeout -k 10 600 bash tools/emulate_split.sh c3 > gpurun_out/r6g_emulate_c3.txt 2>&1 || { cat gpurun_out/r6g_emulate_c3.txt; exit 1; }
cat gpurun_out/r6g_emulate_c3.txt
PT_SMALL_LAUNCH=0 timeout -k 10 600 bash tools/emulate_split.sh c3 > gpurun_out/r6g_emulate_c3_off.txt 2>&1 || { cat gpurun_out/r6g_emulate_c3_off.txt; exit 1; }
cat gpurun_out/r6g_emulate_c3_off.txt
timeout -k 10 600 bash tools/emulate_split.sh c4 > gpurun_out/r6g_emulate_c4.txt 2>&1 || { cat gpurun_out/r6g_emulate_c4.txt; exit 1; }
cat gpurun_out/r6g_emulate_c4.txt
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 600 bash tools/ab.sh c3 3 $L $L,PT_SMALL_LAUNCH=0 > gpurun_out/r6g_ab_c3.txt 2>&1 || { cat gpurun_out/r6g_ab_c3.txt; exit 1; }
cat gpurun_out/r6g_ab_c3.txt
timeout -k 10 600 bash tools/r6_session_c.sh > gpurun_out/r6g_census.txt 2>&1 || { cat gpurun_out/r6g_census.txt; exit 1; }
cat gpurun_out/r6g_census.txt
