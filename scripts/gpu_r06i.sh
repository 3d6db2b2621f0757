#!/bin/bash
# Round 6: kernel traces of the closed-loop tick at 65,536 robots (eager then graph), this
# round's product and round 5's source, to find which kernel the graph replay slows down.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_r5; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06i_$v -o run --output-format csv -- python tools/loop_graph.py 65536 8 $L/$v.so > gpurun_out/r06i_$v.log 2>&1 || { tail -5 gpurun_out/r06i_$v.log; exit 1; }
  grep "^B " gpurun_out/r06i_$v.log
done
echo done
