set -e
mkdir -p gpurun_out
for v in base new5 s20 w6 w6d; do
  echo "== $v"; PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py
done > gpurun_out/img_hash.txt 2>&1
cat gpurun_out/img_hash.txt
timeout -k 10 900 bash tools/ab.sh c3 3 _variants/base.so _variants/new5.so _variants/s20.so _variants/w6.so _variants/w6d.so > gpurun_out/ab_w6_c3.txt 2>&1
cat gpurun_out/ab_w6_c3.txt
timeout -k 10 600 bash tools/ab.sh c3f 2 _variants/base.so _variants/new5.so _variants/w6.so _variants/w6d.so > gpurun_out/ab_w6_c3f.txt 2>&1
cat gpurun_out/ab_w6_c3f.txt
