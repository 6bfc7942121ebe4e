#!/bin/bash
# A/B of the follow-up ray (PT_FOLLOW): GPU suite on the in-tree library, image
# hashes of the three builds, same-session throughput on C3 / framed C3 / C4 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_follow.log 2>&1 || { tail -40 gpurun_out/gpu_tests_follow.log; exit 1; }
tail -1 gpurun_out/gpu_tests_follow.log
{ for v in base follow0 follow; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_follow.txt 2>&1
cat gpurun_out/img_hash_follow.txt
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 3 _variants/base.so _variants/follow0.so _variants/follow.so
  echo "== c3f"; timeout -k 10 600 bash tools/ab.sh c3f 2 _variants/base.so _variants/follow.so
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 _variants/base.so _variants/follow.so
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 2 _variants/base.so _variants/follow.so; } > gpurun_out/ab_follow.txt 2>&1
cat gpurun_out/ab_follow.txt
