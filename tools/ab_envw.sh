set -e
mkdir -p gpurun_out
{ for v in base envw; do echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py; done; } > gpurun_out/img_hash_envw.txt 2>&1
cat gpurun_out/img_hash_envw.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_envw.log 2>&1 || { tail -30 gpurun_out/gpu_tests_envw.log; exit 1; }
tail -1 gpurun_out/gpu_tests_envw.log
{ echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 3 _variants/base.so _variants/envw.so; } > gpurun_out/ab_envw.txt 2>&1
cat gpurun_out/ab_envw.txt
