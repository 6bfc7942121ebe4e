#!/bin/bash
# round 5: eight interleaved queue heads (PT_QUEUE_HEADS=8) vs one, after the
# claim-latency census (profiles/r5/census_claims.txt): C3 5 rounds, C4 / C5 2.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab.sh c3 5 _variants/h1.so _variants/h8.so > gpurun_out/r5aa_ab_c3.txt 2>&1 || { cat gpurun_out/r5aa_ab_c3.txt; exit 1; }
cat gpurun_out/r5aa_ab_c3.txt
timeout -k 10 600 bash tools/ab.sh c4 2 _variants/h1.so _variants/h8.so > gpurun_out/r5aa_ab_c4.txt 2>&1 || { cat gpurun_out/r5aa_ab_c4.txt; exit 1; }
cat gpurun_out/r5aa_ab_c4.txt
timeout -k 10 600 bash tools/ab.sh c5 2 _variants/h1.so _variants/h8.so > gpurun_out/r5aa_ab_c5.txt 2>&1 || { cat gpurun_out/r5aa_ab_c5.txt; exit 1; }
cat gpurun_out/r5aa_ab_c5.txt
