#!/bin/bash
# Round-end style check: GPU parity tests, then the full measurement (bench, kernel trace, PMC).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?
tail -3 gpurun_out/test.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash scripts/gpu_full.sh
