#!/bin/bash
# Round-4 A/B on one box: GPU tests on the product library, then the headline workloads
# (gpu_ab.sh) of the given builds, the one-GPU shard rehearsal, and per-phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
TESTS=0 R=${R:-2} CASES="${CASES:-3:65536 2:65536 2:4096 1:256 1:1024 1:65536}" bash scripts/gpu_ab.sh "$@" || exit 1
for var in "$@"; do
  tag=$(basename $var .so)
  timeout -k 10 300 python tools/shard_times.py $var 5 > gpurun_out/shard_$tag.log 2>&1 || { echo "shard_times failed"; tail -5 gpurun_out/shard_$tag.log; exit 1; }
  echo "shards $tag"; grep "N=" gpurun_out/shard_$tag.log
done
if [ -f $L/libcmpc_stamps.so ]; then
  for c in 1 2; do
    timeout -k 10 120 python tools/stamps.py --config $c --batch 8192 --team 0 --lib $L/libcmpc_stamps.so > gpurun_out/stamps_c$c.txt 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/stamps_c$c.txt; exit 1; }
    cat gpurun_out/stamps_c$c.txt
  done
fi
echo done
