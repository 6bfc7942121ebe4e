#!/bin/bash
# Extra rocprofv3 PMC passes over one bench.py workload (instruction mix, LDS,
# L1/TA behaviour), one counter group per pass, within the per-block limits.
# Usage: tools/profile_deep.sh <workload> [steps]  -> gpurun_out/prof/<pass>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=${1:-c3}
STEPS=${2:-5}
WARM=2; [ "$WL" = c3 ] && WARM=8  # (C3: 8 frames per launch -- whole batches only, as tools/profile_session.sh)
B="python3 bench.py --workload $WL --steps $STEPS --warmup $WARM --no-cpu-baseline --no-extras"
P="rocprofv3 --output-format csv"
I="PT_PIPELINE=0"  # every render alone: counts per launch
exec tools/gpu_session.sh \
  "sq2:120:$I $P --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS -d gpurun_out/prof/sq2 -o sq2 -- $B" \
  "sq3:120:$I $P --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/prof/sq3 -o sq3 -- $B" \
  "tcp:120:$I $P --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/prof/tcp -o tcp -- $B" \
  "tcp2:120:$I $P --pmc TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum -d gpurun_out/prof/tcp2 -o tcp2 -- $B" \
  "ta:120:$I $P --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum -d gpurun_out/prof/ta -o ta -- $B"
