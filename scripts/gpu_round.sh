#!/bin/bash
# One GPU call: parity tests on the product library, A/B of the given variants on the headline
# workloads (scripts/gpu_ab.sh: path.so[@VAR=val,...]), then the one-GPU strong-scaling
# rehearsal of each variant (tools/shard_times.py).
#   usage: [TESTS=1] [R=2] [CASES=...] [SHARDS=1] bash scripts/gpu_round.sh a.so [b.so@VAR=val ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
  rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
fi
TESTS=0 bash scripts/gpu_ab.sh "$@" || exit 1
if [ "${SHARDS:-1}" = "1" ]; then
  for var in "$@"; do
    lib=${var%%@*}; envs=""; [ "$var" != "$lib" ] && envs=${var#*@}
    tag=$(basename $lib .so)$(echo "$envs" | tr -c 'A-Za-z0-9\n' '_' | sed 's/^./_&/')
    echo "shards $tag"
    env ${envs//,/ } timeout -k 10 300 python tools/shard_times.py $lib 5 > gpurun_out/shard_$tag.log 2>&1 || { echo "shard_times failed"; tail -5 gpurun_out/shard_$tag.log; exit 1; }
    cat gpurun_out/shard_$tag.log
  done
fi
echo done
