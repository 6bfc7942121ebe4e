#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
for v in base acc4g; do
  for c in WRITE_SIZE FETCH_SIZE; do
    PT_PIPELINE=0 PT_LIB=_variants/$v.so timeout -s KILL 90 rocprofv3 --output-format csv --pmc $c -d gpurun_out/pmcab/${v}_$c -o p -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
  done
done
echo ok
