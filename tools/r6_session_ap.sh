# Resolve spread over workgroups per tile (PT_RESOLVE_SUBS 1 = one per tile, the old launch): GPU suite, then A/Bs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ap.log 2>&1
rc=$?; tail -n 2 gpurun_out/gpu_tests_ap.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh c3 3 $L,PT_RESOLVE_SUBS=1 $L $L,PT_RESOLVE_SUBS=8 $L,PT_RESOLVE_SUBS=2 || exit $?
bash tools/ab.sh c4 2 $L,PT_RESOLVE_SUBS=1 $L || exit $?
