#!/bin/bash
# Cost model: cfg1 bench under SolverParams overrides (one line per variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "" "--param polish_refine=8" "--param polish_stable=6" "--param polish_stable=1" "--param polish_refine=2" "--param polish_repairs=0"; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 5 --warmup 2 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --latency-batch 0 ${EXTRA} $v > gpurun_out/pv.json 2>gpurun_out/pv.err || { echo "fail $v"; tail -3 gpurun_out/pv.err; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/pv.json'));print('$v|', 'ms %.3f'%a['ms_per_step'], 'iters %.2f max %d'%(a['iters_mean'],a['iters_max']), 'solved %.5f'%a['solved_frac'])"
done
