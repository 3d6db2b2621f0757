#!/bin/bash
# Round 5: the repair budget per polish session under the LDL' build (polish_repairs 6 / 4 / 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc.so@CMPC_PARAMS=polish_repairs=4 $L/libcmpc.so@CMPC_PARAMS=polish_repairs=3 || exit 1
for r in 4 3; do
  CMPC_PARAMS=polish_repairs=$r timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rep$r.log 2>&1 || { tail -5 gpurun_out/shard_rep$r.log; exit 1; }
  echo "== polish_repairs $r"; grep N= gpurun_out/shard_rep$r.log
done
echo done
