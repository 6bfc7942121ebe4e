#!/bin/bash
# round 6, final multi-GPU evidence at the final library: the N-rank bench line
# rehearsed on one GPU (gloo, N = 2 / 4 / 8) and the split shares' one-GPU
# emulation with the exchange through RCCL (PT_DIST_FORCE=1): C3 at 64 and at
# 20 timed frames (the line's defaults: 8 frames per launch), C4 at 10.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
REHEARSE_N="2 4 8" timeout -k 10 700 bash tools/rehearse_dist.sh > gpurun_out/rehearse_final.txt 2>&1 || { cat gpurun_out/rehearse_final.txt; exit 1; }
cat gpurun_out/rehearse_final.txt
PT_DIST_FORCE=1 EMU_STEPS=64 timeout -k 10 700 bash tools/emulate_split.sh c3 > gpurun_out/emulate_c3_rccl_64.txt 2>&1 || { cat gpurun_out/emulate_c3_rccl_64.txt; exit 1; }
cat gpurun_out/emulate_c3_rccl_64.txt
PT_DIST_FORCE=1 EMU_STEPS=20 timeout -k 10 700 bash tools/emulate_split.sh c3 > gpurun_out/emulate_c3_rccl_20.txt 2>&1 || { cat gpurun_out/emulate_c3_rccl_20.txt; exit 1; }
cat gpurun_out/emulate_c3_rccl_20.txt
PT_DIST_FORCE=1 timeout -k 10 700 bash tools/emulate_split.sh c4 > gpurun_out/emulate_c4_rccl.txt 2>&1 || { cat gpurun_out/emulate_c4_rccl.txt; exit 1; }
cat gpurun_out/emulate_c4_rccl.txt
