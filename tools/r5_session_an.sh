#!/bin/bash
# round 5: 1024-slot claims for large frames (PT_CHUNK_BIG=1024) vs 512.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_suite.sh -w "c5:2 c5big:1 c4:2" -o r5an_c1024 _variants/c512.so _variants/c1024.so > /dev/null 2>&1 || { cat gpurun_out/r5an_c1024.txt; exit 1; }
cat gpurun_out/r5an_c1024.txt
