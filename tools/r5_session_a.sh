cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r5_gpu_w8.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/r5_gpu_w8.log | tail -15
if [ $rc -le 1 ]; then
  timeout -k 10 600 bash tools/ab.sh c3 3 _variants/head.so _variants/w4.so _variants/w8.so > gpurun_out/r5_ab_width_c3.txt 2>&1; echo "ab c3 rc=$?"; cat gpurun_out/r5_ab_width_c3.txt
fi
