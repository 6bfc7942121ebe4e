#!/bin/bash
# Host AddressSanitizer + UBSan build of every libptgpu.so source (HIP
# translation units included: -fsanitize applies to HOST code only, each flag
# after -Xarch_host; device code is not instrumented) linked into
# tests/sanitize/gpu_driver.cpp.  build: here (cross-compiles for gfx950);
# run: on the GPU box (tools/sanitize_gpu.sh run).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=_build/asan
if [ "${1:-build}" = build ]; then
  mkdir -p "$OUT"
  SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -fno-omit-frame-pointer"
  INC="-Iinclude -Idsgpuraytracing_amd/csrc"
  objs=()
  for f in dsgpuraytracing_amd/csrc/*.hip dsgpuraytracing_amd/csrc/pt_api.cpp tests/sanitize/gpu_driver.cpp; do
    o="$OUT/$(basename "$f").o"
    hipcc --offload-arch=gfx950 -O1 -g -std=c++17 $SAN $INC -fno-slp-vectorize -x hip -c "$f" -o "$o" &
    objs+=("$o")
  done
  for f in scene_host render_tree exr_io image_out pt_error; do
    o="$OUT/$f.o"
    hipcc -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=all -fno-gpu-sanitize $INC -xc++ -c "dsgpuraytracing_amd/csrc/$f.cpp" -o "$o" &
    objs+=("$o")
  done
  wait
  hipcc --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -o "$OUT/gpu_driver" "${objs[@]}" -lz
  echo "built $OUT/gpu_driver"
else
  export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=0
  export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
  BIG=$(python -c "from dsgpuraytracing_amd import scenes; print(scenes.proxy_path(1))")
  timeout -k 10 300 "$OUT/gpu_driver" assets/CBspheres_lambertian.dae tests/golden/env_sky_64x32.exr "$BIG"
fi
