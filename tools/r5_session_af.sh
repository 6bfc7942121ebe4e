#!/bin/bash
# round 5 final multi-GPU readiness evidence at HEAD (one GPU): the N = 2 / 4 / 8
# C4 tile-split emulation and the gloo/RCCL rehearsal line with efficiencies;
# the drain census of the final kernel.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 400 bash tools/emulate_split.sh c4 > gpurun_out/r5af_emulate_split_c4.txt 2>&1 || { cat gpurun_out/r5af_emulate_split_c4.txt; exit 1; }
cat gpurun_out/r5af_emulate_split_c4.txt
timeout -k 10 600 bash tools/rehearse_dist.sh > gpurun_out/r5af_rehearse.txt 2>&1 || { tail -30 gpurun_out/r5af_rehearse.txt; exit 1; }
tail -5 gpurun_out/r5af_rehearse.txt
