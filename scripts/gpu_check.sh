#!/bin/bash
# GPU parity tests, then one bench headline under a rocprofv3 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -3 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -30; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/test.log | sed 's/ PASSED.*//' | tail -40 > /dev/null
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --aux 0 --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof.log; exit 1; }
  tail -1 gpurun_out/prof.log
fi
echo done
