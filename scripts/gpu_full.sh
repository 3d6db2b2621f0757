#!/bin/bash
# Full measurement: bench (with CPU baseline), rocprofv3 kernel trace, PMC HBM traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 500 python bench.py ${BENCH_ARGS} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --latency-batch 0 --dynamics-steps 0 --warm-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --latency-batch 0 --dynamics-steps 0 --warm-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/pmc_f.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --latency-batch 0 --dynamics-steps 0 --warm-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/pmc_w.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo done
