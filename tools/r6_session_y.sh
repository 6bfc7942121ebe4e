#!/bin/bash
# round 6, session y: kernel + HIP runtime traces of the C3 N = 8 share at the
# default (exchange on the current stream) with RCCL in the loop, to see what
# each render waits for: its hardware queue, its slot's previous resolve, or
# the host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5 --emulate-shard 8 --emulate-rank 0"
PT_DIST_FORCE=1 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace --hip-runtime-trace -d gpurun_out/r6y/ns8 -o ns8 -- $B > gpurun_out/r6y_ns8.log 2>&1
rc=$?; tail -n 2 gpurun_out/r6y_ns8.log; ls gpurun_out/r6y/ns8; exit $rc
