#!/bin/bash
# Careful A/B: cfg1/cfg2 bench, product vs variant, 4 alternations each; prints means.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1
EX="--cpu-seconds 0 --steps 20 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0"
for cfg in 1 2; do
  : > gpurun_out/ab3_$cfg.txt
  for rep in 1 2 3 4; do
    timeout -k 10 120 python bench.py $EX --config $cfg > gpurun_out/a.json 2>/dev/null || exit 1
    timeout -k 10 120 python bench.py $EX --config $cfg --lib $VAR > gpurun_out/b.json 2>/dev/null || exit 1
    python -c "import json;a=json.load(open('gpurun_out/a.json'));b=json.load(open('gpurun_out/b.json'));print(a['value'],b['value'],a['latency_ms_b256'],b['latency_ms_b256'])" >> gpurun_out/ab3_$cfg.txt
  done
  python -c "
import numpy as np;d=np.loadtxt('gpurun_out/ab3_$cfg.txt')
print('cfg$cfg base %.3fM +-%.3f  var %.3fM +-%.3f  ratio %.3f  lat %.3f/%.3f'%(d[:,0].mean()/1e6,d[:,0].std()/1e6,d[:,1].mean()/1e6,d[:,1].std()/1e6,(d[:,1]/d[:,0]).mean(),d[:,2].mean(),d[:,3].mean()))"
done
