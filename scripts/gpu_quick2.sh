#!/bin/bash
# Selected GPU tests (args: pytest -k expression) then a bench line without the CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ${1:+-k "$1"} > gpurun_out/test.log 2>&1
rc=$?
tail -3 gpurun_out/test.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "^E |Error|FAILED|max err" gpurun_out/test.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
