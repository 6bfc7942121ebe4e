#!/bin/bash
# Same-session PMC A/B of library builds / knobs: one rocprofv3 --pmc pass
# (SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES) per arm
# over `bench.py --workload <wl>` with PT_PIPELINE=0 (every launch alone), then
# the render kernel's per-launch averages per arm (tools/pmc_valu_summary.py).
# An arm is "name=lib.so" or "name=lib.so,VAR=v,VAR2=v".
# Usage: tools/pmc_valu.sh <workload> r3=_variants/r3.so new=_variants/new.so,PT_SAMPLE_GROUP=8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=$1; shift
OUT=gpurun_out/pmcvalu_$WL
rm -rf "$OUT"
for arm in "$@"; do
  name=${arm%%=*}; rest=${arm#*=}
  IFS=, read -r lib envs <<< "$rest"
  env PT_PIPELINE=0 PT_LIB="$lib" ${envs//,/ } timeout -s KILL 120 rocprofv3 --output-format csv \
    --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    -d "$OUT/$name" -o sq -- python3 bench.py --workload "$WL" --steps 3 --warmup 1 \
    --no-cpu-baseline --no-extras > /dev/null 2>&1 || { echo "FAILED $name"; exit 3; }
done
python3 tools/pmc_valu_summary.py "$OUT" "$WL"
