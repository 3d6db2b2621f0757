#!/bin/bash
# quick iteration: mfma layout check, parity tests, stamps, bench (+ optional rocprof)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 tools/mfma_layout_check.hip -o /tmp/mfma_check > gpurun_out/mfma.log 2>&1 && timeout -k 10 60 /tmp/mfma_check >> gpurun_out/mfma.log 2>&1
cat gpurun_out/mfma.log
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test.log 2>&1
rc=$?
tail -15 gpurun_out/test.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
timeout -k 10 300 python tools/stamps.py --config 1 > gpurun_out/stamps1.txt 2>&1 || { echo stamps1 failed; cat gpurun_out/stamps1.txt; exit 1; }
timeout -k 10 300 python tools/stamps.py --config 2 > gpurun_out/stamps2.txt 2>&1 || { echo stamps2 failed; cat gpurun_out/stamps2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps1.txt gpurun_out/stamps2.txt
PROF=${PROF:-0} bash scripts/gpu_bench.sh
