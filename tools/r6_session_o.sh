#!/bin/bash
# round 6, session o: render streams 2 and 3 created only when a small launch
# uses them -- whole C3 frame against the round-5 library (tools/ab.sh, 4
# rounds, same box), and the C3 split emulation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 800 bash tools/ab.sh c3 4 _variants/head.so dsgpuraytracing_amd/libptgpu.so > gpurun_out/r6o_ab_head.txt 2>&1 || { cat gpurun_out/r6o_ab_head.txt; exit 1; }
cat gpurun_out/r6o_ab_head.txt
timeout -k 10 600 bash tools/emulate_split.sh c3 > gpurun_out/r6o_emulate_c3.txt 2>&1 || { cat gpurun_out/r6o_emulate_c3.txt; exit 1; }
cat gpurun_out/r6o_emulate_c3.txt
