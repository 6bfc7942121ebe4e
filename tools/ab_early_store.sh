#!/bin/bash
# A/B of the early group store (PT_EARLY_STORE) over the follow-up rays:
# GPU suite on the in-tree library, image hashes, same-session throughput,
# then a launch-knob re-sweep on the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_es.log 2>&1 || { tail -40 gpurun_out/gpu_tests_es.log; exit 1; }
tail -1 gpurun_out/gpu_tests_es.log
{ for v in follow es; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_es.txt 2>&1
cat gpurun_out/img_hash_es.txt
{ echo "== c3"; timeout -k 10 600 bash tools/ab_full.sh c3 3 _variants/follow.so _variants/es.so
  echo "== c3f"; timeout -k 10 600 bash tools/ab_full.sh c3f 2 _variants/follow.so _variants/es.so
  echo "== c4"; timeout -k 10 600 bash tools/ab_full.sh c4 2 _variants/follow.so _variants/es.so
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 2 _variants/follow.so _variants/es.so _variants/es_env0.so; } > gpurun_out/ab_es.txt 2>&1
cat gpurun_out/ab_es.txt
L=_variants/es.so
{ echo "== c3"; timeout -k 10 900 bash tools/ab_full.sh c3 1 $L $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=48 $L,PT_SAMPLE_GROUP=8 $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=12
  echo "== c4"; timeout -k 10 900 bash tools/ab_full.sh c4 1 $L $L,PT_SHADE_BATCH=24 $L,PT_SHADE_BATCH=40 $L,PT_SAMPLE_GROUP=8
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 1 $L $L,PT_SHADE_BATCH=32 $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=56; } > gpurun_out/ab_knobs_es.txt 2>&1
cat gpurun_out/ab_knobs_es.txt
