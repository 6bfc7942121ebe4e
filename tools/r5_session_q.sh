#!/bin/bash
# round 5 final evidence at the current library: GPU suite, smoke, bench lines
# (C3 default with companions and CPU baselines; C4, C5, c5big one-GPU lines).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 1000 bash tools/final_bench.sh > gpurun_out/r5q_final_bench.log 2>&1 || { tail -30 gpurun_out/r5q_final_bench.log; exit 1; }
tail -8 gpurun_out/r5q_final_bench.log
