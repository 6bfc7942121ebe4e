set -e
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
{ echo "== c3"; timeout -k 10 600 bash tools/ab.sh c3 2 $L $L,PT_LEAF_WEIGHT=12 $L,PT_LEAF_WEIGHT=20 $L,PT_LEAF_WEIGHT=24 $L,PT_DRAIN_DIV=2
  echo "== c4"; timeout -k 10 600 bash tools/ab.sh c4 2 $L $L,PT_LEAF_WEIGHT=12 $L,PT_LEAF_WEIGHT=20 $L,PT_DRAIN_DIV=2
  echo "== c5"; timeout -k 10 900 bash tools/ab.sh c5 1 $L $L,PT_LEAF_WEIGHT=12 $L,PT_LEAF_WEIGHT=20 $L,PT_DRAIN_DIV=2; } > gpurun_out/ab_leaf.txt 2>&1
cat gpurun_out/ab_leaf.txt
