#!/bin/bash
# Launch-knob re-sweep after the follow-up rays (shading-round size, sample
# group, leaf weight), same session, in-tree library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
L=dsgpuraytracing_amd/libptgpu.so
{ echo "== c3"; timeout -k 10 900 bash tools/ab_full.sh c3 2 $L $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=48 $L,PT_SAMPLE_GROUP=8 $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=12
  echo "== c4"; timeout -k 10 900 bash tools/ab_full.sh c4 1 $L $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=48 $L,PT_SAMPLE_GROUP=8
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 1 $L $L,PT_SHADE_BATCH=32 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=56 $L,PT_SAMPLE_GROUP=8; } > gpurun_out/ab_knobs_follow.txt 2>&1
cat gpurun_out/ab_knobs_follow.txt
