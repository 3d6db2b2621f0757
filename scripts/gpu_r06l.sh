#!/bin/bash
# Round 6: the closed-loop graph replay at 65,536 robots with and without the next replay queued
# behind the running one (a device synchronisation after every tick), this round's product vs
# round 5's source; a kernel trace of the synchronised graph replay of the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_r5 libcmpc; do
  echo "== $v"
  timeout -k 10 200 python -u tools/loop_graph.py 65536 12 $L/$v.so eager,graph,eagersync,graphsync 2>&1 | grep "^B " || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06l_sync -o run --output-format csv -- python tools/loop_graph.py 65536 8 $L/libcmpc.so graphsync,graph > gpurun_out/r06l_sync.log 2>&1 || { tail -5 gpurun_out/r06l_sync.log; exit 1; }
grep "^B " gpurun_out/r06l_sync.log
echo done
