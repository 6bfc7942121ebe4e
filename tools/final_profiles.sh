# rocprofv3 sessions (kernel traces + PMC passes) for C3, C4, C5 and C5big at the current library
# (then: python tools/profile_summary.py c3 profiles/<r> gpurun_out/prof_c3 "" 8; the others with 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/profile_session.sh c3 16 gpurun_out/prof_c3 && \
bash tools/profile_session.sh c4 4 gpurun_out/prof_c4 && \
bash tools/profile_session.sh c5 3 gpurun_out/prof_c5 && \
bash tools/profile_session.sh c5big 3 gpurun_out/prof_c5big
