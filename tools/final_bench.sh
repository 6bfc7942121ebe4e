# End-of-round evidence at the current library: GPU suite, smoke, bench lines (C3 default with companions and
# CPU baselines; C4 and C5 single-GPU lines).  Every GPU step under its own limit; stop after a hang/fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -n 3 gpurun_out/smoke.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_c3_default.jsonl 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4_1gpu.jsonl 2> gpurun_out/bench_c4.err || exit $?
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_1gpu.jsonl 2> gpurun_out/bench_c5.err || exit $?
timeout -k 10 300 python bench.py --workload c5big --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5big_1gpu.jsonl 2> gpurun_out/bench_c5big.err || exit $?
for f in c3_default c4_1gpu c5_1gpu c5big_1gpu; do tail -n 1 gpurun_out/bench_$f.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['bound'], r['frac'], r.get('frac_isolated'), r.get('pmc_stale'))"; done
