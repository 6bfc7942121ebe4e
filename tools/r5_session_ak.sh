#!/bin/bash
# round 5: 512-slot claims for busy / large frames (PT_CHUNK_MAX=512, c512) vs 256 (fix).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_suite.sh -H "fix c512" -w "c3:3 c4:1 c5:2" -o r5ak_c512 _variants/fix.so _variants/c512.so > /dev/null 2>&1 || { cat gpurun_out/r5ak_c512.txt; exit 1; }
cat gpurun_out/r5ak_c512.txt
