#!/bin/bash
# round 6, session j: the LDS treelet with nodes padded to 144 B in LDS
# (wg4t40p / wg4t20p) against base and the unpadded wg4t45: correctness,
# counters (lone launches), and tools/ab.sh on C3 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in wg4t40p wg4t20p; do
  PT_LIB=_variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread \
    -k "near_exact or deterministic or resident_grid or claim_size or drain_helpers or deep_bvh or tri_only" > gpurun_out/r6j_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6j_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6j_tests_$v.log)"
  PT_LIB=_variants/$v.so timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6j_hash_$v.txt || exit 1
done
PT_LIB=_variants/base.so timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6j_hash_base.txt || exit 1
for v in wg4t40p wg4t20p; do diff -q gpurun_out/r6j_hash_base.txt gpurun_out/r6j_hash_$v.txt && echo "$v: image hashes identical to base"; done
timeout -k 10 300 bash tools/pmc_pass.sh c3 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" base=_variants/base.so wg4t45=_variants/wg4t45.so wg4t40p=_variants/wg4t40p.so wg4t20p=_variants/wg4t20p.so || exit 1
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum" base=_variants/base.so wg4t40p=_variants/wg4t40p.so || exit 1
B=_variants/base.so
timeout -k 10 600 bash tools/ab.sh c3 4 $B _variants/wg4t40p.so _variants/wg4t20p.so > gpurun_out/r6j_ab_c3.txt 2>&1 || { cat gpurun_out/r6j_ab_c3.txt; exit 1; }
cat gpurun_out/r6j_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c5 1 $B _variants/wg4t40p.so > gpurun_out/r6j_ab_c5.txt 2>&1 || { cat gpurun_out/r6j_ab_c5.txt; exit 1; }
cat gpurun_out/r6j_ab_c5.txt
