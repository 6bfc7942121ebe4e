#!/bin/bash
# round 5 (re-entry): GPU suite + bench line on the current defaults, then the
# same-session A/B of the round-5 switches against the round-4 library:
#   r4  = round-4 HEAD (a642b50)      cur = defaults (nearest-first order, split ballots)
#   o0  = PT_NODE_ORDER=0 (sort net)  b0  = PT_BALLOT_SPLIT=0
#   s4  = PT_SUM_WORDS=4 (16-B sums)  w8  = PT_NODE_WIDTH=8
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5g_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5g_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r5g_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5g_bench.err; exit 1; }
tail -c 1500 gpurun_out/r5g_bench.json; echo
timeout -k 10 900 bash tools/ab.sh c3 3 _variants/r4.so _variants/cur.so _variants/o0.so _variants/b0.so _variants/s4.so > gpurun_out/r5g_ab_c3.txt 2>&1 || { cat gpurun_out/r5g_ab_c3.txt; exit 1; }
cat gpurun_out/r5g_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c5 1 _variants/r4.so _variants/cur.so _variants/o0.so _variants/b0.so _variants/s4.so > gpurun_out/r5g_ab_c5.txt 2>&1 || { cat gpurun_out/r5g_ab_c5.txt; exit 1; }
cat gpurun_out/r5g_ab_c5.txt
timeout -k 10 300 bash tools/pmc_valu.sh c3 r4=_variants/r4.so cur=_variants/cur.so o0=_variants/o0.so b0=_variants/b0.so > gpurun_out/r5g_pmc_valu_c3.txt 2>&1 || { cat gpurun_out/r5g_pmc_valu_c3.txt; exit 1; }
cat gpurun_out/r5g_pmc_valu_c3.txt
timeout -k 10 400 bash tools/pmc_pass.sh c5 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" cur=_variants/cur.so s4=_variants/s4.so > gpurun_out/r5g_pmc_sums_c5.txt 2>&1 || { cat gpurun_out/r5g_pmc_sums_c5.txt; exit 1; }
cat gpurun_out/r5g_pmc_sums_c5.txt
