# round 5: node step child order (nearest-first + slot pushes) and single-compare ballots
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/ab_full_c3.jsonl
AB_FULL=1 timeout -k 10 600 bash tools/ab.sh c3 3 _variants/w4.so _variants/o1.so _variants/b1.so _variants/ob.so > gpurun_out/r5_ab_order_c3.txt 2>&1 || exit 1
cat gpurun_out/r5_ab_order_c3.txt
timeout -k 10 300 bash tools/ab.sh c3f 1 _variants/w4.so _variants/ob.so || exit 1
timeout -k 10 400 bash tools/ab.sh c5 1 _variants/w4.so _variants/ob.so || exit 1
timeout -k 10 300 bash tools/pmc_valu.sh c3 w4=_variants/w4.so ob=_variants/ob.so || exit 1
# 16-B group-sum records (PT_SUM_WORDS=4) against 12-B ones: write traffic and L2 hit rate
timeout -k 10 400 bash tools/ab.sh c3 2 _variants/ob.so _variants/s4.so || exit 1
timeout -k 10 400 bash tools/ab.sh c5 1 _variants/ob.so _variants/s4.so || exit 1
timeout -k 10 300 bash tools/pmc_pass.sh c3 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ob=_variants/ob.so s4=_variants/s4.so || exit 1
timeout -k 10 400 bash tools/pmc_pass.sh c5 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ob=_variants/ob.so s4=_variants/s4.so || exit 1
