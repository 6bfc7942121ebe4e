#!/bin/bash
# round 5: GPU suite on the new defaults (sorting-network child order, env
# records as two vector loads, triangle-only kernel), A/B against round 4 and
# the mixed kernel (PT_NO_TRI_ONLY), and the instruction-cost probes
# (PT_PROBE_*: +32 SALU / VALU per traversal iteration, +128 per shading round).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5h_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5h_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5h_gpu_tests.log
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c3 3 _variants/r4.so _variants/new.so _variants/new.so,PT_NO_TRI_ONLY=1 > gpurun_out/r5h_ab_c3.txt 2>&1 || { cat gpurun_out/r5h_ab_c3.txt; exit 1; }
cat gpurun_out/r5h_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c3 1 _variants/new.so _variants/ts32.so _variants/tv32.so _variants/ss128.so _variants/sv128.so > gpurun_out/r5h_probes_c3.txt 2>&1 || { cat gpurun_out/r5h_probes_c3.txt; exit 1; }
cat gpurun_out/r5h_probes_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 2 _variants/r4.so _variants/new.so _variants/new.so,PT_NO_TRI_ONLY=1 > gpurun_out/r5h_ab_c5.txt 2>&1 || { cat gpurun_out/r5h_ab_c5.txt; exit 1; }
cat gpurun_out/r5h_ab_c5.txt
timeout -k 10 200 bash tools/pmc_valu.sh c3 new=_variants/new.so mixed=_variants/new.so,PT_NO_TRI_ONLY=1 > gpurun_out/r5h_pmc_valu_c3.txt 2>&1 || { cat gpurun_out/r5h_pmc_valu_c3.txt; exit 1; }
cat gpurun_out/r5h_pmc_valu_c3.txt
