#!/bin/bash
# round 5: runtime knobs re-swept on the new kernel (leaf weight, shading-round
# size, drain divisor) -- C3 2 rounds, C5 and C4 1 round.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
L=_variants/head.so
timeout -k 10 500 bash tools/ab.sh c3 2 $L $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=16 $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_DRAIN_DIV=2 > gpurun_out/r5l_knobs_c3.txt 2>&1 || { cat gpurun_out/r5l_knobs_c3.txt; exit 1; }
cat gpurun_out/r5l_knobs_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 1 $L $L,PT_LEAF_WEIGHT=12 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=56 > gpurun_out/r5l_knobs_c5.txt 2>&1 || { cat gpurun_out/r5l_knobs_c5.txt; exit 1; }
cat gpurun_out/r5l_knobs_c5.txt
timeout -k 10 300 bash tools/ab.sh c4 1 $L $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=16 $L,PT_SHADE_BATCH=40 > gpurun_out/r5l_knobs_c4.txt 2>&1 || { cat gpurun_out/r5l_knobs_c4.txt; exit 1; }
cat gpurun_out/r5l_knobs_c4.txt
