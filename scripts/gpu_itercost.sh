#!/bin/bash
# Per-ADMM-iteration cost: pure ADMM (no polish, no rho adaptation) at two iteration caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for mi in 10 50; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 5 --warmup 2 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --latency-batch 0 --param polish_stable=100000 --param adaptive_rho_interval=0 --param max_iter=$mi > gpurun_out/ic.json 2>gpurun_out/ic.err || { echo fail; tail -3 gpurun_out/ic.err; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/ic.json'));print('max_iter $mi', 'ms %.3f'%a['ms_per_step'], 'iters %.2f'%a['iters_mean'])"
done
