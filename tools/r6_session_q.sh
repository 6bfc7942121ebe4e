#!/bin/bash
# round 6, session q: kernel traces (timestamps per dispatch) of the C3 split
# shares (one-GPU emulation, rank 0, N = 8 and 2) and of the whole C3 frame,
# 60 pipelined frames each, to see where a share's 0.24-0.30 ms per frame goes
# (render overlap, resolve / exchange kernels, gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P="rocprofv3 --output-format csv --kernel-trace"
B="python3 bench.py --workload c3 --no-cpu-baseline --no-extras --steps 60 --warmup 5"
timeout -k 10 240 $P -d gpurun_out/r6q/emu8 -o emu8 -- $B --emulate-shard 8 --emulate-rank 0 > gpurun_out/r6q_emu8.log 2>&1 && \
timeout -k 10 240 $P -d gpurun_out/r6q/emu2 -o emu2 -- $B --emulate-shard 2 --emulate-rank 0 > gpurun_out/r6q_emu2.log 2>&1 && \
timeout -k 10 240 $P -d gpurun_out/r6q/whole -o whole -- $B > gpurun_out/r6q_whole.log 2>&1
rc=$?
tail -n 1 gpurun_out/r6q_emu8.log gpurun_out/r6q_emu2.log gpurun_out/r6q_whole.log | cut -c1-300
exit $rc
