#!/bin/bash
# Builds libptgpu.so variants for A/B runs: each argument "name:FLAGS" gives
# _variants/name.so built with PT_HIPCC_FLAGS=FLAGS; the tree's own library is
# rebuilt unchanged afterwards.  Usage: tools/variants.sh "base:" "x:-DPT_FOO=0"
cd "$(dirname "$0")/.." || exit 2
mkdir -p _variants
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  PT_HIPCC_FLAGS="$flags" python -c "from dsgpuraytracing_amd import build; build.build(force=True)" || exit 1
  cp dsgpuraytracing_amd/libptgpu.so "_variants/$name.so"
done
python -c "from dsgpuraytracing_amd import build; build.build(force=True)"
