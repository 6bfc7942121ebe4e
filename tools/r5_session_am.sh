#!/bin/bash
# round 5 final evidence at HEAD: GPU suite, smoke, bench lines, then the rocprofv3 summaries.
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
bash tools/r5_session_q.sh || exit 1
bash tools/r5_session_r.sh
