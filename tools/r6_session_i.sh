#!/bin/bash
# round 6, session i: counters of the LDS treelet (wg4t45) against the round-6
# library (base) on C3, lone launches (PT_PIPELINE=0): texture-addresser load,
# vector-memory reads, instruction counts, waiting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum" base=_variants/base.so wg4=_variants/wg4.so wg4t45=_variants/wg4t45.so || exit 1
timeout -k 10 300 bash tools/pmc_pass.sh c3 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" base=_variants/base.so wg4=_variants/wg4.so wg4t45=_variants/wg4t45.so || exit 1
