# round 5: the direction-free Trav (w4 = this tree at PT_NODE_WIDTH=4) against HEAD of round 4
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab.sh c3 5 _variants/head.so _variants/w4.so > gpurun_out/r5_ab_dfree_c3.txt 2>&1 || exit 1
cat gpurun_out/r5_ab_dfree_c3.txt
timeout -k 10 400 bash tools/ab.sh c3f 2 _variants/head.so _variants/w4.so > gpurun_out/r5_ab_dfree_c3f.txt 2>&1 || exit 1
cat gpurun_out/r5_ab_dfree_c3f.txt
timeout -k 10 500 bash tools/ab.sh c5 2 _variants/head.so _variants/w4.so > gpurun_out/r5_ab_dfree_c5.txt 2>&1 || exit 1
cat gpurun_out/r5_ab_dfree_c5.txt
