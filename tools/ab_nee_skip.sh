set -e
mkdir -p gpurun_out
{ for v in base nee; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_nee.txt 2>&1
cat gpurun_out/img_hash_nee.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_nee.log 2>&1 || { tail -30 gpurun_out/gpu_tests_nee.log; exit 1; }
tail -1 gpurun_out/gpu_tests_nee.log
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 3 _variants/base.so _variants/nee.so
  echo "== c3f"; timeout -k 10 600 bash tools/ab.sh c3f 2 _variants/base.so _variants/nee.so
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 _variants/base.so _variants/nee.so
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 2 _variants/base.so _variants/nee.so; } > gpurun_out/ab_nee_skip.txt 2>&1
cat gpurun_out/ab_nee_skip.txt
