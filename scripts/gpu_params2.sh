#!/bin/bash
# cfg1/cfg2 bench under a list of SolverParams overrides (args: one quoted override set each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in 1 2; do
for v in "$@"; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --config $cfg --steps 6 --warmup 2 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 --latency-batch 0 $v > gpurun_out/pv.json 2>gpurun_out/pv.err || { echo "fail $v"; tail -3 gpurun_out/pv.err; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/pv.json'));print('cfg$cfg $v|', 'ms %.3f'%a['ms_per_step'], 'iters %.2f max %d'%(a['iters_mean'],a['iters_max']), 'solved %.5f'%a['solved_frac'])"
done; done
