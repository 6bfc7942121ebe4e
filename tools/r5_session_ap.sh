#!/bin/bash
# round 5 final: the deep PMC passes (instruction mix, LDS, L1 / TA) of the final C3 kernel.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out; rm -f gpurun_out/session.log; rm -rf gpurun_out/prof
timeout -k 10 900 bash tools/profile_deep.sh c3 5 > gpurun_out/r5ap_deep.log 2>&1 || { tail -30 gpurun_out/r5ap_deep.log; exit 1; }
grep "rc=" gpurun_out/session.log | tail -6
