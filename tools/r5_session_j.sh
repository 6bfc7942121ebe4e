#!/bin/bash
# round 5: step-selection simplification (PT_SEL_SIMPLE) and local waits for
# stack-spill loads (PT_SPILL_WAIT) A/B on C3 / C5; the 8-wide node (w8) on
# C4 and c5big; the one-GPU emulation of the multi-GPU C4 tile split.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
AB_FULL=1 timeout -k 10 500 bash tools/ab.sh c3 3 _variants/head.so _variants/sf.so _variants/sel0.so _variants/sw0.so > gpurun_out/r5j_ab_c3.txt 2>&1 || { cat gpurun_out/r5j_ab_c3.txt; exit 1; }
cat gpurun_out/r5j_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 1 _variants/head.so _variants/sf.so > gpurun_out/r5j_ab_c5.txt 2>&1 || { cat gpurun_out/r5j_ab_c5.txt; exit 1; }
cat gpurun_out/r5j_ab_c5.txt
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c4 1 _variants/head.so _variants/w8.so > gpurun_out/r5j_ab_c4.txt 2>&1 || { cat gpurun_out/r5j_ab_c4.txt; exit 1; }
cat gpurun_out/r5j_ab_c4.txt
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c5big 1 _variants/head.so _variants/w8.so > gpurun_out/r5j_ab_c5big.txt 2>&1 || { cat gpurun_out/r5j_ab_c5big.txt; exit 1; }
cat gpurun_out/r5j_ab_c5big.txt
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TCC_HIT_sum TCC_MISS_sum" head=_variants/head.so w8=_variants/w8.so > gpurun_out/r5j_l2_c3.txt 2>&1 || { cat gpurun_out/r5j_l2_c3.txt; exit 1; }
cat gpurun_out/r5j_l2_c3.txt
PT_LIB=_variants/head.so timeout -k 10 400 bash tools/emulate_split.sh c4 > gpurun_out/r5j_emulate_split_c4.txt 2>&1 || { cat gpurun_out/r5j_emulate_split_c4.txt; exit 1; }
cat gpurun_out/r5j_emulate_split_c4.txt
