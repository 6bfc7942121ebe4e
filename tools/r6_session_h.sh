#!/bin/bash
# round 6, session h: 4-wave workgroups (wg4) and the LDS treelet of the top of
# the render tree (wg4t21 / wg4t45: 21 / 45 nodes of the level-by-level order
# in the workgroup's LDS; a node step reads a treelet node from LDS, the
# others from global memory) against the round-6 library (base).  First a
# near-exact / bit-identity check of each variant (PT_LIB), then tools/ab.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in wg4 wg4t21 wg4t45; do
  PT_LIB=_variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread \
    -k "near_exact or deterministic or resident_grid or claim_size or drain_helpers or deep_bvh or tri_only" > gpurun_out/r6h_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6h_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6h_tests_$v.log)"
  PT_LIB=_variants/$v.so timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6h_hash_$v.txt || exit 1
done
PT_LIB=_variants/base.so timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6h_hash_base.txt || exit 1
for v in wg4 wg4t21 wg4t45; do diff -q gpurun_out/r6h_hash_base.txt gpurun_out/r6h_hash_$v.txt && echo "$v: image hashes identical to base"; done
B=_variants/base.so; V1=_variants/wg4.so; V2=_variants/wg4t21.so; V3=_variants/wg4t45.so
AB_FULL=1 timeout -k 10 600 bash tools/ab.sh c3 3 $B $V1 $V2 $V3 > gpurun_out/r6h_ab_c3.txt 2>&1 || { cat gpurun_out/r6h_ab_c3.txt; exit 1; }
cat gpurun_out/r6h_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c3f 2 $B $V1 $V2 $V3 > gpurun_out/r6h_ab_c3f.txt 2>&1 || { cat gpurun_out/r6h_ab_c3f.txt; exit 1; }
cat gpurun_out/r6h_ab_c3f.txt
timeout -k 10 600 bash tools/ab.sh c4 1 $B $V1 $V2 $V3 > gpurun_out/r6h_ab_c4.txt 2>&1 || { cat gpurun_out/r6h_ab_c4.txt; exit 1; }
cat gpurun_out/r6h_ab_c4.txt
timeout -k 10 600 bash tools/ab.sh c5 1 $B $V1 $V2 $V3 > gpurun_out/r6h_ab_c5.txt 2>&1 || { cat gpurun_out/r6h_ab_c5.txt; exit 1; }
cat gpurun_out/r6h_ab_c5.txt
