#!/bin/bash
# round 6, session k: GPU suite + smoke at the committed library, the default
# bench line, and 64-slot claims for the whole C3 frame (one frame alone and
# pipelined; tools/ab.sh, 3 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r6k_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6k_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r6k_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k_smoke.log 2>&1 || { cat gpurun_out/r6k_smoke.log; exit 1; }
tail -1 gpurun_out/r6k_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r6k_bench_c3.jsonl 2> gpurun_out/r6k_bench_c3.err || { tail -20 gpurun_out/r6k_bench_c3.err; exit 1; }
tail -n 1 gpurun_out/r6k_bench_c3.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d['config']; print('c3', d['value'], d['ms_per_step'], 'single', c['single_frame_ms'], 'iso', r['isolated_kernel_ms'], 'frac', r['frac'], 'frac_kernel', r['frac_kernel'], 'stale', r['pmc_stale'], 'traced', d['traced_samples_per_s_M'], 'single_Mrays', d['single_frame_Mrays'])"
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 600 bash tools/ab.sh c3 3 $L $L,PT_CHUNK_SLOTS=64 > gpurun_out/r6k_ab_chunk64.txt 2>&1 || { cat gpurun_out/r6k_ab_chunk64.txt; exit 1; }
cat gpurun_out/r6k_ab_chunk64.txt
