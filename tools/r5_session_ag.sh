#!/bin/bash
# round 5 final: the C3 profile again (PT_PIPELINE=0 launches now take the
# latency-mode claim), then the multi-GPU readiness evidence at HEAD.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out; rm -f gpurun_out/session.log
timeout -k 10 600 bash tools/profile_session.sh c3 5 gpurun_out/prof_c3 > gpurun_out/r5ag_prof_c3.log 2>&1 || { tail -30 gpurun_out/r5ag_prof_c3.log; exit 1; }
grep "rc=" gpurun_out/session.log | tail -6
bash tools/r5_session_af.sh
