#!/bin/bash
# round 5: tail claims (the last slots per lane dealt 64 at a time from a
# second queue head: PT_TAIL_CLAIMS / PT_TAIL_SLOTS) and the cheaper
# triangle predicate -- GPU suite on the new default, A/B on C3 / C5 / C4.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5m_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5m_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5m_gpu_tests.log
N=_variants/new.so
timeout -k 10 500 bash tools/ab.sh c3 3 _variants/head.so $N $N,PT_TAIL_SLOTS=0 $N,PT_TAIL_SLOTS=2 > gpurun_out/r5m_ab_c3.txt 2>&1 || { cat gpurun_out/r5m_ab_c3.txt; exit 1; }
cat gpurun_out/r5m_ab_c3.txt
timeout -k 10 300 bash tools/ab.sh c5 1 _variants/head.so $N $N,PT_TAIL_SLOTS=0 > gpurun_out/r5m_ab_c5.txt 2>&1 || { cat gpurun_out/r5m_ab_c5.txt; exit 1; }
cat gpurun_out/r5m_ab_c5.txt
timeout -k 10 300 bash tools/ab.sh c4 1 _variants/head.so $N $N,PT_TAIL_SLOTS=0 > gpurun_out/r5m_ab_c4.txt 2>&1 || { cat gpurun_out/r5m_ab_c4.txt; exit 1; }
cat gpurun_out/r5m_ab_c4.txt
