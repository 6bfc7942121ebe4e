# round 5: node-width A/B completion + node order / ballots / 16-B sums A/Bs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_c5.jsonl gpurun_out/ab_full_c3.jsonl
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
AB_FULL=1 timeout -k 10 600 bash tools/ab.sh c3 3 _variants/w4.so _variants/o1.so _variants/b1.so _variants/ob.so > gpurun_out/r5_ab_order_c3.txt 2>&1 || exit 1
cat gpurun_out/r5_ab_order_c3.txt
timeout -k 10 300 bash tools/ab.sh c3f 1 _variants/w4.so _variants/ob.so || exit 1
timeout -k 10 400 bash tools/ab.sh c5 1 _variants/w4.so _variants/ob.so || exit 1
timeout -k 10 300 bash tools/pmc_valu.sh c3 w4=_variants/w4.so ob=_variants/ob.so || exit 1
timeout -k 10 400 bash tools/ab.sh c3 2 _variants/ob.so _variants/s4.so || exit 1
timeout -k 10 400 bash tools/ab.sh c5 1 _variants/ob.so _variants/s4.so || exit 1
timeout -k 10 300 bash tools/pmc_pass.sh c3 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ob=_variants/ob.so s4=_variants/s4.so || exit 1
timeout -k 10 400 bash tools/pmc_pass.sh c5 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ob=_variants/ob.so s4=_variants/s4.so || exit 1
