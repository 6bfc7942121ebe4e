#!/bin/bash
# rocprofv3 passes over one bench.py workload on the GPU box (one counter
# group per pass; --pmc never combined with runtime/sys traces).
# Usage: tools/profile_session.sh <workload> [steps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=${1:-c3}
STEPS=${2:-5}
B="python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline --no-extras"
P="rocprofv3 --output-format csv"
rm -rf gpurun_out/prof
exec tools/gpu_session.sh \
  "kt:300:$P --kernel-trace --stats -d gpurun_out/prof/kt -o kt -- $B" \
  "fetch:300:$P --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o fetch -- $B" \
  "write:300:$P --pmc WRITE_SIZE -d gpurun_out/prof/write -o write -- $B" \
  "sq:300:$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/prof/sq -o sq -- $B" \
  "tcc:300:$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/tcc -o tcc -- $B"
