#!/bin/bash
# round 5: the 512-slot claim A/B, then the final evidence at HEAD (GPU suite,
# smoke, bench lines).
cd "$GRAFT_REPO_ROOT" || exit 2; mkdir -p gpurun_out
bash tools/r5_session_ak.sh || exit 1
bash tools/r5_session_q.sh
