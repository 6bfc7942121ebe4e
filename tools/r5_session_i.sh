#!/bin/bash
# round 5: LDS stack fast paths (PT_STACK_FAST, wave-uniform: pushes / pops
# without per-lane spill branches) -- GPU suite on the default, A/B against
# the same build without them (nosf) and the 8-wide node (w8) on C3 / C5,
# launch counters (AB_FULL) and SQ instruction / wait counters.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_c3.jsonl gpurun_out/ab_full_c5.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5i_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5i_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5i_gpu_tests.log
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c3 3 _variants/sf.so _variants/nosf.so _variants/w8.so > gpurun_out/r5i_ab_c3.txt 2>&1 || { cat gpurun_out/r5i_ab_c3.txt; exit 1; }
cat gpurun_out/r5i_ab_c3.txt
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c5 1 _variants/sf.so _variants/nosf.so _variants/w8.so > gpurun_out/r5i_ab_c5.txt 2>&1 || { cat gpurun_out/r5i_ab_c5.txt; exit 1; }
cat gpurun_out/r5i_ab_c5.txt
timeout -k 10 300 bash tools/pmc_valu.sh c3 sf=_variants/sf.so nosf=_variants/nosf.so w8=_variants/w8.so > gpurun_out/r5i_pmc_valu_c3.txt 2>&1 || { cat gpurun_out/r5i_pmc_valu_c3.txt; exit 1; }
cat gpurun_out/r5i_pmc_valu_c3.txt
