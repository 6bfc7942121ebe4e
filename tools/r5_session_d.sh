# round 5: the node-width A/B completed -- L2 hit, C4 / c5big throughput, C5 launch counters
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_c5.jsonl
timeout -k 10 300 bash tools/pmc_pass.sh c3 "TCC_HIT_sum TCC_MISS_sum" w4=_variants/w4.so w8=_variants/w8.so || exit 1
timeout -k 10 300 bash tools/ab.sh c4 2 _variants/w4.so _variants/w8.so || exit 1
AB_FULL=1 timeout -k 10 400 bash tools/ab.sh c5 1 _variants/w4.so _variants/w8.so || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_full_c5.jsonl"):
    d = json.loads(l); c = d["line"]["launch_counters"]
    print(d["variant"], {k: c[k] for k in ("node_visits", "tri_tests", "sphere_tests", "wave_trav_steps", "leaf_steps", "wave_rounds")})
PY
timeout -k 10 600 bash tools/ab.sh c5big 1 _variants/w4.so _variants/w8.so || exit 1
