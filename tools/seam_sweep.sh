set -e
mkdir -p gpurun_out
DAE=$(python3 -c "from dsgpuraytracing_amd import scenes; print(scenes.C1_DAE)")
for b in 16 32 64 128 256 512 1024; do
  echo -n "batch $b: "
  PT_TILE_BATCH=$b timeout -k 10 120 ./dsgpuraytracing_amd/seam_bench "$DAE" 1024 1024 64 8 5
done > gpurun_out/seam_sweep.txt 2>&1
cat gpurun_out/seam_sweep.txt
