set -e
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 2 $L $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=36 $L,PT_SHADE_BATCH=32
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 $L $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=36
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 2 $L $L,PT_SHADE_BATCH=40 $L,PT_SHADE_BATCH=36; } > gpurun_out/ab_batch.txt 2>&1
cat gpurun_out/ab_batch.txt
