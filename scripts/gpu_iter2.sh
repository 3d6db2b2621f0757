#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -3 gpurun_out/test.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/test.log; exit 1; }
timeout -k 10 300 python tools/find_hard.py gpurun_out/hard.json > gpurun_out/hard.log 2>&1 || { cat gpurun_out/hard.log; exit 1; }
cat gpurun_out/hard.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_w.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_f.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
