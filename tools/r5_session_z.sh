#!/bin/bash
# round 5: drain census with queue-claim latency (PT_CENSUS=1 builds): the one
# queue head, tail claims, eight heads; C3 and C5 (lone launches).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
for lib in census census_tail census_h8; do
  for wl in c3 c5; do
    echo "## $lib $wl"
    PT_LIB=_variants/$lib.so timeout -k 10 300 python tools/wave_trace.py --census --workload $wl 2>gpurun_out/r5z_err.log || { tail -20 gpurun_out/r5z_err.log; exit 1; }
  done
done
