#!/bin/bash
# round 5: non-temporal group-sum stores (PT_NT_SUMS=1, nt) vs plain (tt) on the
# large scenes, with the L2 counters (L2 hit >= 0.80 on C5).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
PMC_PASSES="WRITE_SIZE FETCH_SIZE TCC_HIT_sum,TCC_MISS_sum" timeout -k 10 600 bash tools/pmc_ab.sh c5 _variants/tt.so _variants/nt.so > gpurun_out/r5ah_pmc_c5.txt 2>&1 || { cat gpurun_out/r5ah_pmc_c5.txt; exit 1; }
cat gpurun_out/r5ah_pmc_c5.txt
timeout -k 10 600 bash tools/ab.sh c5 2 _variants/tt.so _variants/nt.so > gpurun_out/r5ah_ab_c5.txt 2>&1 || { cat gpurun_out/r5ah_ab_c5.txt; exit 1; }
cat gpurun_out/r5ah_ab_c5.txt
timeout -k 10 600 bash tools/ab.sh c5big 1 _variants/tt.so _variants/nt.so > gpurun_out/r5ah_ab_c5big.txt 2>&1 || { cat gpurun_out/r5ah_ab_c5big.txt; exit 1; }
cat gpurun_out/r5ah_ab_c5big.txt
timeout -k 10 600 bash tools/ab.sh c3 2 _variants/tt.so _variants/nt.so > gpurun_out/r5ah_ab_c3.txt 2>&1 || { cat gpurun_out/r5ah_ab_c3.txt; exit 1; }
cat gpurun_out/r5ah_ab_c3.txt
