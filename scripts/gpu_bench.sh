#!/bin/bash
# bench + rocprofv3 kernel trace on one GPU (used via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
CPUS=${CPUS:-0}
timeout -k 10 400 python bench.py --steps $STEPS --warmup 2 --cpu-seconds $CPUS ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; exit 1; }
cat gpurun_out/bench.json
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
