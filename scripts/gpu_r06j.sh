#!/bin/bash
# Round 6: the closed-loop graph replay at 65,536 robots against ROCr's scratch handling (the
# r06i traces: after the solve, the replayed tick's small kernels stretch 6 -> 45 us every ~58 us
# with this round's library only; its solve kernels need 48 / 96 B of scratch per lane, round 5's
# 32 / 72 B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
L=convex-mpc-unitree-go2_amd/cmpc/lib
run() {
  echo "== $1 ${2:-}"
  env $2 timeout -k 10 200 python -u tools/loop_graph.py 65536 12 $L/$1.so 2>&1 | grep "^B " || exit 1
}
run libcmpc
run libcmpc HSA_NO_SCRATCH_RECLAIM=1
run libcmpc HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0
run libcmpc HSA_NO_SCRATCH_THREAD_LIMITER=1
run libcmpc HSA_SCRATCH_SINGLE_LIMIT=4294967296
run libcmpc_r5
echo done
