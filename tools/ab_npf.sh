#!/bin/bash
# Same-session A/B: vertex-normal prefetch into L1 at a new nearest hit (npf,
# LDS-DMA into a dummy), shading-phase wave priority + iterative-ILP scheduling
# of the environment-light build (p1e), and both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
set -e
PT_LIB=_variants/npf_p1e.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_npf.log 2>&1 || { tail -40 gpurun_out/gpu_tests_npf.log; exit 1; }
tail -1 gpurun_out/gpu_tests_npf.log
{ echo "== c3"; timeout -k 10 900 bash tools/ab_full.sh c3 3 _variants/es.so _variants/npf.so _variants/p1e.so _variants/npf_p1e.so
  echo "== c3f"; timeout -k 10 900 bash tools/ab_full.sh c3f 2 _variants/es.so _variants/npf.so _variants/p1e.so _variants/npf_p1e.so
  echo "== c4"; timeout -k 10 900 bash tools/ab_full.sh c4 2 _variants/es.so _variants/npf.so _variants/p1e.so _variants/npf_p1e.so
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 2 _variants/es.so _variants/npf.so _variants/p1e.so _variants/npf_p1e.so; } > gpurun_out/ab_npf.txt 2>&1
cat gpurun_out/ab_npf.txt
