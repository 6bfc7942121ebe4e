#!/bin/bash
# round 5: c5big A/B (head / 8-wide / compressed 4-wide node), C3 L2 hit rates
# of the three, and the one-GPU emulation of the multi-GPU C4 tile split.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c5big 1 _variants/head.so _variants/w8.so _variants/nc.so > gpurun_out/r5k_ab_c5big.txt 2>&1 || { cat gpurun_out/r5k_ab_c5big.txt; exit 1; }
cat gpurun_out/r5k_ab_c5big.txt
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TCC_HIT_sum TCC_MISS_sum" head=_variants/head.so w8=_variants/w8.so nc=_variants/nc.so > gpurun_out/r5k_l2_c3.txt 2>&1 || { cat gpurun_out/r5k_l2_c3.txt; exit 1; }
cat gpurun_out/r5k_l2_c3.txt
PT_LIB=_variants/head.so timeout -k 10 400 bash tools/emulate_split.sh c4 > gpurun_out/r5k_emulate_split_c4.txt 2>&1 || { cat gpurun_out/r5k_emulate_split_c4.txt; exit 1; }
cat gpurun_out/r5k_emulate_split_c4.txt
# round-5 evidence at this library: C3 rocprofv3 kernel traces + PMC passes, the default bench line
timeout -k 10 900 bash tools/profile_session.sh c3 5 gpurun_out/prof_c3 > gpurun_out/r5k_prof_c3.log 2>&1 || { tail -30 gpurun_out/r5k_prof_c3.log; exit 1; }
grep "rc=" gpurun_out/session.log | tail -8
timeout -k 10 400 python bench.py > gpurun_out/r5k_bench_c3.jsonl 2> gpurun_out/r5k_bench_c3.err || { tail -20 gpurun_out/r5k_bench_c3.err; exit 1; }
tail -n 1 gpurun_out/r5k_bench_c3.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], d['config'].get('single_frame_ms'), r['bound'], r['frac'], r.get('frac_isolated'), r.get('pmc_stale'))"
