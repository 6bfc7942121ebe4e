#!/bin/bash
# One same-session A/B experiment on the GPU box (replaces round 3's per-
# experiment tools/ab_*.sh scripts):
#   -t LIB       first run the GPU suite against LIB (PT_LIB) and stop if it fails
#   -H "A B"     image hashes (tools/img_hash.py) of _variants/A.so, _variants/B.so ...
#   -w "c3:3 c4:2"  workloads and rounds for tools/ab.sh (AB_FULL=1 for the counters)
#   -o NAME      write everything to gpurun_out/NAME.txt as well
# then the variants ("lib.so" or "lib.so,VAR=val,...") as tools/ab.sh takes them.
# Usage: tools/ab_suite.sh -t _variants/new.so -H "base new" -w "c3:3 c3f:2 c4:2 c5:2" -o ab_new \
#          _variants/base.so _variants/new.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
TESTLIB=""; HASH=""; WLS="c3:2"; OUT=""
while getopts "t:H:w:o:" o; do
  case $o in t) TESTLIB=$OPTARG ;; H) HASH=$OPTARG ;; w) WLS=$OPTARG ;; o) OUT=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
LOG=gpurun_out/${OUT:-ab_suite}.txt
: > "$LOG"
if [ -n "$TESTLIB" ]; then
  PT_LIB=$TESTLIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "gpurun_out/gpu_tests_${OUT:-ab_suite}.log" 2>&1
  rc=$?; tail -n 1 "gpurun_out/gpu_tests_${OUT:-ab_suite}.log" | tee -a "$LOG"
  [ $rc -eq 0 ] || exit $rc
fi
for v in $HASH; do
  echo "== hash $v" | tee -a "$LOG"
  PT_LIB=_variants/$v.so timeout -k 10 200 python3 tools/img_hash.py 2>&1 | tee -a "$LOG"
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
done
for spec in $WLS; do
  wl=${spec%%:*}; rounds=${spec#*:}
  echo "== $wl" | tee -a "$LOG"
  timeout -k 10 1200 bash tools/ab.sh "$wl" "$rounds" "$@" 2>&1 | tee -a "$LOG"
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
done
