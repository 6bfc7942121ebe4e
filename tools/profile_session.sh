#!/bin/bash
# rocprofv3 passes over one bench.py workload on the GPU box (one counter
# group per pass; --pmc never combined with runtime/sys traces).  The PMC
# passes and the second kernel trace run with PT_PIPELINE=0 (every render
# alone on the GPU), so per-launch counts and durations belong to one kernel.
# Usage: tools/profile_session.sh <workload> [steps] [out]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=${1:-c3}
STEPS=${2:-5}
OUT=${3:-gpurun_out/prof}
# (C3 renders 8 frames per launch: whole batches only, so every timed launch
# the passes count is an 8-frame one -- tools/profile_summary.py <wl> <out> <prof> "" 8)
WARM=2; [ "$WL" = c3 ] && WARM=8
B="python3 bench.py --workload $WL --steps $STEPS --warmup $WARM --no-cpu-baseline --no-extras"
P="rocprofv3 --output-format csv"
I="PT_PIPELINE=0"
rm -rf "$OUT"
exec tools/gpu_session.sh \
  "kt_$WL:300:$P --kernel-trace --stats -d $OUT/kt -o kt -- $B" \
  "kt_iso_$WL:300:$I $P --kernel-trace --stats -d $OUT/kt_iso -o kt_iso -- $B" \
  "fetch_$WL:300:$I $P --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- $B" \
  "write_$WL:300:$I $P --pmc WRITE_SIZE -d $OUT/write -o write -- $B" \
  "sq_$WL:300:$I $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/sq -o sq -- $B" \
  "tcc_$WL:300:$I $P --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o tcc -- $B"
