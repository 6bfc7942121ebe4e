#!/bin/bash
# round 6, session ac: frame batches as the strong split's default: GPU suite,
# the N = 2 / 4 rehearsal, C3 split emulation (defaults: 8 frames per launch,
# RCCL in the loop, 64 frames), the N = 1 line's frame_batch field.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ac_gpu_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r6ac_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
REHEARSE_N="2 4" timeout -k 10 500 bash tools/rehearse_dist.sh || exit 1
PT_DIST_FORCE=1 EMU_STEPS=64 timeout -k 10 400 bash tools/emulate_split.sh c3 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r6ac_n1.jsonl 2>gpurun_out/r6ac_n1.err || exit 1
tail -n 1 gpurun_out/r6ac_n1.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n1', d['value'], d['ms_per_step'], d['config']['frames_per_launch'], d.get('frame_batch'))"
