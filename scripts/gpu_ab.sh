#!/bin/bash
# A/B: tests on the product library, then cfg1/cfg2 bench of the product vs a variant library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${1:-convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_wpe1.so}
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/test.log | head -20; exit 1; }
for cfg in 1 2; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --config $cfg > gpurun_out/ab_base_$cfg.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --cpu-seconds 0 --config $cfg --lib $VAR > gpurun_out/ab_var_$cfg.json 2>/dev/null || exit 1
  python -c "import json;a=json.load(open('gpurun_out/ab_base_$cfg.json'));b=json.load(open('gpurun_out/ab_var_$cfg.json'));print('cfg$cfg base %.0f var %.0f  lat %.2f/%.2f ms'%(a['value'],b['value'],a['latency_ms_b256'],b['latency_ms_b256']))"
done
