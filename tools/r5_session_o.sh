#!/bin/bash
# round 5: resolve with 16-B loads, second version (three loads = four groups
# per step, 28 VGPRs: co-resident with the next render's waves) vs the old one.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab.sh c3 3 _variants/new.so _variants/rw0.so _variants/new.so,PT_PIPELINE=0 _variants/rw0.so,PT_PIPELINE=0 > gpurun_out/r5o_ab_c3.txt 2>&1 || { cat gpurun_out/r5o_ab_c3.txt; exit 1; }
cat gpurun_out/r5o_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c4 1 _variants/new.so _variants/rw0.so _variants/new.so,PT_PIPELINE=0 _variants/rw0.so,PT_PIPELINE=0 > gpurun_out/r5o_ab_c4.txt 2>&1 || { cat gpurun_out/r5o_ab_c4.txt; exit 1; }
cat gpurun_out/r5o_ab_c4.txt
timeout -k 10 300 bash tools/ab.sh c5 1 _variants/new.so _variants/rw0.so > gpurun_out/r5o_ab_c5.txt 2>&1 || { cat gpurun_out/r5o_ab_c5.txt; exit 1; }
cat gpurun_out/r5o_ab_c5.txt
