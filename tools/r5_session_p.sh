#!/bin/bash
# round 5: wave priorities of the two phases (s_setprio): shading 2 / traversal 0
# (default) vs traversal raised (0/2, 1/2) vs none (0/0).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab.sh c3 3 _variants/new.so _variants/pt2.so _variants/p00.so _variants/p11.so > gpurun_out/r5p_ab_c3.txt 2>&1 || { cat gpurun_out/r5p_ab_c3.txt; exit 1; }
cat gpurun_out/r5p_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 1 _variants/new.so _variants/pt2.so _variants/p00.so > gpurun_out/r5p_ab_c5.txt 2>&1 || { cat gpurun_out/r5p_ab_c5.txt; exit 1; }
cat gpurun_out/r5p_ab_c5.txt
timeout -k 10 300 bash tools/ab.sh c4 1 _variants/new.so _variants/pt2.so _variants/p00.so > gpurun_out/r5p_ab_c4.txt 2>&1 || { cat gpurun_out/r5p_ab_c4.txt; exit 1; }
cat gpurun_out/r5p_ab_c4.txt
