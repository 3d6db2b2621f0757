#!/bin/bash
# Per-instance anatomy of the config-3 shards (N = 1 and 8): start/duration (times build) and
# iterations/factorizations/cycles (counts build); then an A/B of the given variant libraries
# on the N = 8 shard rehearsal and the config-3 headline.
#   usage: bash scripts/gpu_anatomy.sh [variant.so ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/anat
export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 240 python -u tools/shard_anatomy.py times gpurun_out/anat/cfg3 1 8 > gpurun_out/anat/times.log 2>&1 || { echo "times failed"; tail -5 gpurun_out/anat/times.log; exit 1; }
timeout -k 10 240 python -u tools/shard_anatomy.py counts gpurun_out/anat/cfg3 1 8 > gpurun_out/anat/counts.log 2>&1 || { echo "counts failed"; tail -5 gpurun_out/anat/counts.log; exit 1; }
for lib in $L/libcmpc.so "$@"; do
  tag=$(basename $lib .so)
  timeout -k 10 240 python -u tools/shard_times.py $lib 5 > gpurun_out/anat/shards_$tag.log 2>&1 || { echo "shards $tag failed"; tail -5 gpurun_out/anat/shards_$tag.log; exit 1; }
  tail -4 gpurun_out/anat/shards_$tag.log
done
echo done
