#!/bin/bash
# round 5: GPU suite after the device-independent sample grouping; the N-rank
# bench flow rehearsed on one GPU (gloo; every rank on cuda:0: the strong
# companions' efficiency field, NOT scaling evidence -- the ranks share one GPU).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5t_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5t_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5t_gpu_tests.log
timeout -k 10 900 bash tools/rehearse_dist.sh > gpurun_out/r5t_rehearse.txt 2>&1 || { tail -30 gpurun_out/r5t_rehearse.txt; exit 1; }
cat gpurun_out/r5t_rehearse.txt
