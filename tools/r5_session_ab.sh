#!/bin/bash
# round 5: claim size with eight queue heads (PT_CHUNK_SLOTS knob): C3 64 / 128
# (default) / 256; C5 128 / 256 (default).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 900 bash tools/ab.sh c3 4 $L $L,PT_CHUNK_SLOTS=64 $L,PT_CHUNK_SLOTS=256 > gpurun_out/r5ab_ab_c3.txt 2>&1 || { cat gpurun_out/r5ab_ab_c3.txt; exit 1; }
cat gpurun_out/r5ab_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c5 2 $L $L,PT_CHUNK_SLOTS=128 > gpurun_out/r5ab_ab_c5.txt 2>&1 || { cat gpurun_out/r5ab_ab_c5.txt; exit 1; }
cat gpurun_out/r5ab_ab_c5.txt
