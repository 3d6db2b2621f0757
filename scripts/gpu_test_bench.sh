#!/bin/bash
# parity tests, then bench + rocprof (used via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test.log 2>&1
rc=$?
tail -5 gpurun_out/test.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
bash scripts/gpu_bench.sh
