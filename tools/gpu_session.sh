#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box.  Each step has its own time
# limit; a step that times out, aborts or segfaults ends the session (no GPU
# work after a fault).  Ordinary failures (exit 1, e.g. a failing test) do not.
# Usage: tools/gpu_session.sh "<name>:<seconds>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done
