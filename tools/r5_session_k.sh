#!/bin/bash
# round 5: c5big A/B (head / 8-wide / compressed 4-wide node), C3 L2 hit rates
# of the three, and the one-GPU emulation of the multi-GPU C4 tile split.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c5big 1 _variants/head.so _variants/w8.so _variants/nc.so > gpurun_out/r5k_ab_c5big.txt 2>&1 || { cat gpurun_out/r5k_ab_c5big.txt; exit 1; }
cat gpurun_out/r5k_ab_c5big.txt
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TCC_HIT_sum TCC_MISS_sum" head=_variants/head.so w8=_variants/w8.so nc=_variants/nc.so > gpurun_out/r5k_l2_c3.txt 2>&1 || { cat gpurun_out/r5k_l2_c3.txt; exit 1; }
cat gpurun_out/r5k_l2_c3.txt
PT_LIB=_variants/head.so timeout -k 10 400 bash tools/emulate_split.sh c4 > gpurun_out/r5k_emulate_split_c4.txt 2>&1 || { cat gpurun_out/r5k_emulate_split_c4.txt; exit 1; }
cat gpurun_out/r5k_emulate_split_c4.txt
