#!/bin/bash
# Same-session PMC A/B of environment configurations of the same library:
# one rocprofv3 --pmc pass (SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU
# SQ_BUSY_CYCLES) per arm over `bench.py --workload <wl>`.
# Usage: tools/pmc_ab_env.sh <workload> <name>=<VAR=v,VAR2=v> ...
#   -> gpurun_out/pmcab/<name>/sq_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
WL=$1; shift
for arm in "$@"; do
  name=${arm%%=*}; envs=${arm#*=}
  env ${envs//,/ } timeout -s KILL 90 rocprofv3 --output-format csv \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES \
    -d "gpurun_out/pmcab/$name" -o sq -- python3 bench.py --workload "$WL" --steps 5 --warmup 2 \
    --no-cpu-baseline --no-extras > /dev/null 2>&1 || { echo "FAILED $name"; exit 3; }
  echo "done $name"
done
