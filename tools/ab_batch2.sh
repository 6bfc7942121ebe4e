set -e
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 2 $L,PT_SHADE_BATCH=36 $L,PT_SHADE_BATCH=32 $L,PT_SHADE_BATCH=28 $L,PT_SHADE_BATCH=24
  echo "== c3f"; timeout -k 10 600 bash tools/ab.sh c3f 2 $L $L,PT_SHADE_BATCH=36 $L,PT_SHADE_BATCH=32 $L,PT_SHADE_BATCH=28
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 $L,PT_SHADE_BATCH=36 $L,PT_SHADE_BATCH=32 $L,PT_SHADE_BATCH=28
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 2 $L $L,PT_SHADE_BATCH=56 $L,PT_SHADE_BATCH=64; } > gpurun_out/ab_batch2.txt 2>&1
cat gpurun_out/ab_batch2.txt
