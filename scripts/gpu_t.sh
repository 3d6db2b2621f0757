#!/bin/bash
# quick: GPU parity tests only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -3 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/test.log | head -20; exit 1; }
