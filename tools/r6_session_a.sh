#!/bin/bash
# round 6, session a: GPU suite on the pruned kernel (+ the >= 256-spp parity
# tests), image hashes of the round-5 library (_variants/head.so) against the
# pruned one, and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r6a_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r6a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6a_gpu_tests.log
timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6a_hash_new.txt || exit 1
PT_LIB=_variants/head.so timeout -k 10 300 python tools/img_hash.py > gpurun_out/r6a_hash_head.txt || exit 1
diff gpurun_out/r6a_hash_head.txt gpurun_out/r6a_hash_new.txt && echo "IMAGE HASHES IDENTICAL"
timeout -k 10 400 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail -20 gpurun_out/r6a_bench.err; exit 1; }
tail -c 3000 gpurun_out/r6a_bench.json
