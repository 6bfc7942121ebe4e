#!/bin/bash
# round 5 final evidence: rocprofv3 kernel traces + PMC passes for C3 / C4 / C5 / c5big.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out; rm -f gpurun_out/session.log
timeout -k 10 1100 bash tools/final_profiles.sh > gpurun_out/r5r_final_profiles.log 2>&1 || { tail -30 gpurun_out/r5r_final_profiles.log; exit 1; }
grep "rc=" gpurun_out/session.log | tail -24
