#!/bin/bash
# round 6, final multi-GPU evidence at the final library: the N-rank bench line
# rehearsed on one GPU (gloo, N = 2 / 4 / 8) and the split shares' one-GPU
# emulation with the exchange through RCCL (PT_DIST_FORCE=1), C3 and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
REHEARSE_N="2 4 8" timeout -k 10 700 bash tools/rehearse_dist.sh > gpurun_out/rehearse_final.txt 2>&1 || { cat gpurun_out/rehearse_final.txt; exit 1; }
cat gpurun_out/rehearse_final.txt
PT_DIST_FORCE=1 timeout -k 10 400 bash tools/emulate_split.sh c3 > gpurun_out/emulate_c3_rccl.txt 2>&1 || { cat gpurun_out/emulate_c3_rccl.txt; exit 1; }
cat gpurun_out/emulate_c3_rccl.txt
PT_DIST_FORCE=1 timeout -k 10 400 bash tools/emulate_split.sh c4 > gpurun_out/emulate_c4_rccl.txt 2>&1 || { cat gpurun_out/emulate_c4_rccl.txt; exit 1; }
cat gpurun_out/emulate_c4_rccl.txt
