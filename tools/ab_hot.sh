#!/bin/bash
# Same-session A/B of a candidate build (_variants/hot.so _variants/hot_all.so) against HEAD (_variants/base.so):
# GPU suite on the candidate, image hashes of both, throughput with launch counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
set -e
PT_LIB=_variants/hot_all.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_hot.log 2>&1 || { tail -40 gpurun_out/gpu_tests_hot.log; exit 1; }
tail -1 gpurun_out/gpu_tests_hot.log
{ for v in base hot hot_all; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_hot.txt 2>&1
cat gpurun_out/img_hash_hot.txt
{ echo "== c3"; timeout -k 10 900 bash tools/ab_full.sh c3 3 _variants/base.so _variants/hot.so _variants/hot_all.so
  echo "== c3f"; timeout -k 10 900 bash tools/ab_full.sh c3f 2 _variants/base.so _variants/hot.so _variants/hot_all.so
  echo "== c4"; timeout -k 10 900 bash tools/ab_full.sh c4 2 _variants/base.so _variants/hot.so _variants/hot_all.so
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 2 _variants/base.so _variants/hot.so _variants/hot_all.so; } > gpurun_out/ab_hot.txt 2>&1
cat gpurun_out/ab_hot.txt
