#!/bin/bash
# A/B without tests: cfg1/cfg2 bench, product vs variant, alternated twice (noise check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1
for rep in 1 2; do for cfg in 1 2; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --config $cfg --steps 10 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/a.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py --cpu-seconds 0 --config $cfg --steps 10 --warm-steps 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 --lib $VAR > gpurun_out/b.json 2>/dev/null || exit 1
  python -c "import json;a=json.load(open('gpurun_out/a.json'));b=json.load(open('gpurun_out/b.json'));print('cfg$cfg base %.0f var %.0f (%+.1f%%)  lat %.2f/%.2f'%(a['value'],b['value'],100*(b['value']/a['value']-1),a['latency_ms_b256'],b['latency_ms_b256']))"
done; done
