#!/bin/bash
# round 6, session c: the node-step census (pt_stats.node_census, STATS build)
# on C3, framed C3, C4 and C5: wave-uniform node steps (scalar-load candidates)
# and node steps inside the top BVH4 levels (LDS-treelet candidates).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for wl in c3 c3f c4 c5; do
  timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r6c_$wl.json 2> gpurun_out/r6c_$wl.err || { tail -20 gpurun_out/r6c_$wl.err; exit 1; }
  tail -n 1 gpurun_out/r6c_$wl.json | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['launch_counters']; n=c['node_census']
w,u,cov,l,t2w,t2l,t3w,t3l=n
print('$wl', 'wave node steps', w, 'uniform', round(u/max(w,1),4), 'lanes at first lane node', round(cov/max(l,1),4),
      'lanes/step', round(l/max(w,1),2), 'top2 steps', round(t2w/max(w,1),4), 'top2 lanes', round(t2l/max(l,1),4),
      'top3 steps', round(t3w/max(w,1),4), 'top3 lanes', round(t3l/max(l,1),4), 'node_visits', c['node_visits'], 'wave_trav_steps', c['wave_trav_steps'], 'leaf_steps', c['leaf_steps'])"
done
