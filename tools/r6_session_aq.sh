# A/B arm: 8-wide nodes of fp32 boxes (greedy collapse of the GPU tree, two DNodes per node; -DPT_W8=1)
# at 4 waves per SIMD (126 VGPRs, no scratch; at 5 waves it spills 96 B per lane), against the shipped
# library and the shipped kernel at 4 waves per SIMD.  Parity first (near-exact at full size).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=dsgpuraytracing_amd/libptgpu.so
W8=_variants/libptgpu_w8_4w.so
B4=_variants/libptgpu_4w.so
PT_LIB=$W8 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread \
  -k "near_exact or sampled_tiles or eight_way" > gpurun_out/gpu_tests_aq_w8.log 2>&1
rc=$?; tail -n 3 gpurun_out/gpu_tests_aq_w8.log; [ $rc -le 1 ] || exit $rc
AB_FULL=1 bash tools/ab.sh c3 3 $L $W8 $B4 || exit $?
bash tools/ab.sh c4 1 $L $W8 || exit $?
bash tools/ab.sh c5 1 $L $W8 || exit $?
