#!/bin/bash
# A/B of speculative traversal (postponed leaves, PT_POSTPONE): GPU suite on the
# postponing build, image hashes, same-session throughput with launch counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
set -e
mkdir -p gpurun_out
PT_LIB=_variants/pp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_pp.log 2>&1 || { tail -40 gpurun_out/gpu_tests_pp.log; exit 1; }
tail -1 gpurun_out/gpu_tests_pp.log
{ for v in es pp; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_pp.txt 2>&1
cat gpurun_out/img_hash_pp.txt
{ echo "== c3"; timeout -k 10 600 bash tools/ab_full.sh c3 3 _variants/es.so _variants/pp.so
  echo "== c3f"; timeout -k 10 600 bash tools/ab_full.sh c3f 2 _variants/es.so _variants/pp.so
  echo "== c4"; timeout -k 10 600 bash tools/ab_full.sh c4 2 _variants/es.so _variants/pp.so
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 2 _variants/es.so _variants/pp.so _variants/pp_env0.so _variants/w4.so; } > gpurun_out/ab_pp.txt 2>&1
cat gpurun_out/ab_pp.txt
