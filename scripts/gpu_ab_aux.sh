#!/bin/bash
# A/B of the auxiliary kernels (dynamics, traj): bench with --steps 1 and each library variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 3 --warm-steps 0 --dynamics-steps 20 --tick-steps 20 --latency-batch 0 --lib $lib > gpurun_out/ab_aux.json 2>gpurun_out/ab_aux.err || { echo "bench failed $lib"; tail gpurun_out/ab_aux.err; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/ab_aux.json'));print('$lib', 'dyn %.4f ms %.3f'%(a['dynamics']['ms_per_step'],a['dynamics']['roofline']['frac']), 'traj %.4f ms %.3f'%(a['tick']['ms_per_step'],a['tick']['roofline']['frac']), 'tick/s %.3g'%a['tick']['full_tick_per_s'])"
done
