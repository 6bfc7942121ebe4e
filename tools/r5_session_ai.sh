#!/bin/bash
# round 5 final: drain census of the final kernel (PT_CENSUS=1 build), C3 lone
# launch and C3 with PT_NO_HELPERS, C5.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
for wl in c3 c5; do
  echo "## census $wl"
  PT_LIB=_variants/census.so timeout -k 10 300 python tools/wave_trace.py --census --workload $wl 2>gpurun_out/r5ai_err.log || { tail -20 gpurun_out/r5ai_err.log; exit 1; }
done
echo "## census c3 PT_NO_HELPERS=1"
PT_NO_HELPERS=1 PT_LIB=_variants/census.so timeout -k 10 300 python tools/wave_trace.py --census --workload c3 2>gpurun_out/r5ai_err.log || { tail -20 gpurun_out/r5ai_err.log; exit 1; }
