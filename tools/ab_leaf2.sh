set -e
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 2 $L $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=10 $L,PT_LEAF_WEIGHT=12
  echo "== c3f"; timeout -k 10 600 bash tools/ab.sh c3f 2 $L $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=10 $L,PT_LEAF_WEIGHT=12
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 $L $L,PT_LEAF_WEIGHT=8 $L,PT_LEAF_WEIGHT=10 $L,PT_LEAF_WEIGHT=12
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 1 $L $L,PT_LEAF_WEIGHT=10 $L,PT_LEAF_WEIGHT=12; } > gpurun_out/ab_leaf2.txt 2>&1
cat gpurun_out/ab_leaf2.txt
