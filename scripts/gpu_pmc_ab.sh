#!/bin/bash
# A/B of two library builds on one box: GPU tests on the product library, the HBM write traffic
# of the config-3 headline launch (PMC WRITE_SIZE, its own pass), headline workloads alternating,
# and the strong-scaling shard times (tools/shard_times.py).
#   usage: bash scripts/gpu_pmc_ab.sh a.so b.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcab; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
for lib in "$@"; do
  v=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcab/$v -o run -- python bench.py --aux 0 --config 3 --steps 2 --warmup 1 --lib $lib > gpurun_out/pmcab/$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
TESTS=0 R=${R:-2} CASES=${CASES:-"1:65536 3:65536 2:4096 3:8192"} bash scripts/gpu_ab.sh "$@" || exit 1
for lib in "$@"; do
  v=$(basename $lib .so)
  timeout -k 5 150 python tools/shard_times.py $lib > gpurun_out/shard_$v.txt 2>&1 || { echo "shards $v failed"; exit 1; }
done
echo done
