#!/bin/bash
# Round 5: launch order of the two register classes under the LDL' build (NC <= 128 first at
# every size: CMPC_HEAVY_FIRST=0) and 3 instead of 6 face downdates per factorization
# (libcmpc_dd3.so) -- A/B and shard rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
TESTS=0 R=2 CASES="3:65536 2:65536 2:4096 3:16384" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc.so@CMPC_HEAVY_FIRST=0 $L/libcmpc_dd3.so || exit 1
timeout -k 10 300 python -u tools/shard_times.py $L/libcmpc_dd3.so 5 > gpurun_out/shard_dd3.log 2>&1 || { tail -5 gpurun_out/shard_dd3.log; exit 1; }
echo "== dd3"; grep N= gpurun_out/shard_dd3.log
CMPC_HEAVY_FIRST=0 timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_hf0.log 2>&1 || { tail -5 gpurun_out/shard_hf0.log; exit 1; }
echo "== heavy_first 0"; grep N= gpurun_out/shard_hf0.log
echo done
