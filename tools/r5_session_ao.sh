#!/bin/bash
# round 5: shading-round size and leaf weight re-checked on the final queue (C3).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 900 bash tools/ab.sh c3 3 $L $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=16 > gpurun_out/r5ao_knobs.txt 2>&1 || { cat gpurun_out/r5ao_knobs.txt; exit 1; }
cat gpurun_out/r5ao_knobs.txt
