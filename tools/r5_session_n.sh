#!/bin/bash
# round 5: resolve with 16-B vector loads (PT_RESOLVE_WIDE) -- GPU suite on the
# new default; A/B of the resolve (pipelined and lone, PT_PIPELINE=0) on C3,
# C4 and C5; image hashes of both builds must agree (same summation order).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5n_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5n_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5n_gpu_tests.log
timeout -k 10 300 bash tools/ab.sh c3 3 _variants/new.so _variants/rw0.so _variants/new.so,PT_PIPELINE=0 _variants/rw0.so,PT_PIPELINE=0 > gpurun_out/r5n_ab_c3.txt 2>&1 || { cat gpurun_out/r5n_ab_c3.txt; exit 1; }
cat gpurun_out/r5n_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c4 1 _variants/new.so _variants/rw0.so _variants/new.so,PT_PIPELINE=0 _variants/rw0.so,PT_PIPELINE=0 > gpurun_out/r5n_ab_c4.txt 2>&1 || { cat gpurun_out/r5n_ab_c4.txt; exit 1; }
cat gpurun_out/r5n_ab_c4.txt
timeout -k 10 300 bash tools/ab.sh c5 1 _variants/new.so _variants/rw0.so > gpurun_out/r5n_ab_c5.txt 2>&1 || { cat gpurun_out/r5n_ab_c5.txt; exit 1; }
cat gpurun_out/r5n_ab_c5.txt
for v in new rw0; do PT_LIB=_variants/$v.so timeout -k 10 200 python tools/img_hash.py > gpurun_out/r5n_hash_$v.txt 2>&1 || { cat gpurun_out/r5n_hash_$v.txt; exit 1; }; done
cmp gpurun_out/r5n_hash_new.txt gpurun_out/r5n_hash_rw0.txt && echo "image hashes identical"; cat gpurun_out/r5n_hash_new.txt | tail -5
