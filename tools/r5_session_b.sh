# round 5: width A/B counters (launch counters, PMC VALU/SALU/wait) and knob sweep for the 8-wide node
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_c3.jsonl
AB_FULL=1 timeout -k 10 300 bash tools/ab.sh c3 1 _variants/w4.so _variants/w8.so || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_full_c3.jsonl"):
    d = json.loads(l); print(d["variant"], json.dumps(d["line"]["launch_counters"]))
PY
timeout -k 10 300 bash tools/pmc_valu.sh c3 w4=_variants/w4.so w8=_variants/w8.so || exit 1
timeout -k 10 600 bash tools/ab.sh c3 2 _variants/w8.so,PT_LEAF_WEIGHT=8 _variants/w8.so,PT_LEAF_WEIGHT=16 _variants/w8.so,PT_LEAF_WEIGHT=24 _variants/w8.so,PT_SHADE_BATCH=24 _variants/w8.so,PT_SHADE_BATCH=48 || exit 1
timeout -k 10 400 bash tools/ab.sh c5 1 _variants/w4.so _variants/w8.so || exit 1
