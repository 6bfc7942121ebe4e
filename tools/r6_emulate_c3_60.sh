cd "${GRAFT_REPO_ROOT}" || exit 2
PT_DIST_FORCE=1 EMU_STEPS=60 timeout -k 10 400 bash tools/emulate_split.sh c3
