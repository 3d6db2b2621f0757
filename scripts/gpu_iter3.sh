#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -3 gpurun_out/test.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/test.log; exit 1; }
timeout -k 10 300 python tools/find_hard.py gpurun_out/hard.json > gpurun_out/hard.log 2>&1 || { cat gpurun_out/hard.log; exit 1; }
cat gpurun_out/hard.log
timeout -k 10 300 python tools/stamps.py --config 1 > gpurun_out/stamps1.txt 2>&1 && timeout -k 10 300 python tools/stamps.py --config 2 > gpurun_out/stamps2.txt 2>&1 && grep -v amdgpu.ids gpurun_out/stamps1.txt gpurun_out/stamps2.txt
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --cpu-seconds 0 --config 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { tail gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
