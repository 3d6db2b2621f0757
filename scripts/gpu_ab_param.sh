#!/bin/bash
# cfg throughput of SolverParams overrides over several workload seeds (one build).
# usage: CFG=2 bash scripts/gpu_ab_param.sh "" "polish_stable=2" "alpha=1.7"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
EX="--cpu-seconds 0 --steps 10 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 --latency-batch 0 --config ${CFG:-2}"
for seed in 11 22 33 44 55; do
  line="seed $seed"
  for par in "$@"; do
    pa=""; for kv in $par; do pa="$pa --param $kv"; done
    timeout -k 10 120 python bench.py $EX --seed-offset $seed $pa > gpurun_out/v.json 2>/dev/null || exit 1
    line="$line $(python -c "import json;a=json.load(open('gpurun_out/v.json'));print('%.3f/%.2f/%.3f'%(a['value']/1e6,a['iters_mean'],a['solved_frac']))")"
  done
  echo $line
done
