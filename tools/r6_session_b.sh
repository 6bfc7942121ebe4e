#!/bin/bash
# round 6, session b: the N > 1 default rehearsed (gloo, every rank on one GPU),
# the one-GPU emulation of the C3 strong split at N = 2/4/8 (tools/emulate_split.sh c3),
# the exchange's on-device cost (tools/exchange_cost.py), and the rocprofv3 session
# of the pruned kernel on C3 (PMC summary re-stamped with the new device-code sha).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 bash tools/emulate_split.sh c3 > gpurun_out/r6b_emulate_c3.txt 2>&1 || { cat gpurun_out/r6b_emulate_c3.txt; exit 1; }
cat gpurun_out/r6b_emulate_c3.txt
timeout -k 10 300 python tools/exchange_cost.py > gpurun_out/r6b_exchange_cost.txt 2>&1 || { cat gpurun_out/r6b_exchange_cost.txt; exit 1; }
cat gpurun_out/r6b_exchange_cost.txt
timeout -k 10 900 bash tools/rehearse_dist.sh > gpurun_out/r6b_rehearse.txt 2>&1 || { cat gpurun_out/r6b_rehearse.txt; exit 1; }
cat gpurun_out/r6b_rehearse.txt
timeout -k 10 900 bash tools/profile_session.sh c3 5 gpurun_out/prof_c3 > gpurun_out/r6b_prof.log 2>&1 || { tail -30 gpurun_out/r6b_prof.log; exit 1; }
tail -5 gpurun_out/r6b_prof.log
timeout -k 10 600 python tools/silhouette_samples.py --workload c5 --tile 800,416 > gpurun_out/r6b_silhouette_c5.txt 2>&1 || { tail -20 gpurun_out/r6b_silhouette_c5.txt; exit 1; }
tail -15 gpurun_out/r6b_silhouette_c5.txt
