#!/bin/bash
# Same-session A/B of build options on the early-store kernel: wave priority
# raised for the shading phase (prio1) or for traversal (prio2), FMA
# contraction within expressions only (-ffp-contract=on), the iterative-ILP
# scheduler for the environment-light build (env_ilp, C5 only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
{ echo "== c3"; timeout -k 10 900 bash tools/ab_full.sh c3 2 _variants/es.so _variants/prio1.so _variants/prio2.so _variants/contract_on.so
  echo "== c4"; timeout -k 10 900 bash tools/ab_full.sh c4 2 _variants/es.so _variants/prio1.so _variants/prio2.so _variants/contract_on.so
  echo "== c5"; timeout -k 10 900 bash tools/ab_full.sh c5 2 _variants/es.so _variants/prio1.so _variants/prio2.so _variants/contract_on.so _variants/env_ilp.so; } > gpurun_out/ab_misc.txt 2>&1
cat gpurun_out/ab_misc.txt
