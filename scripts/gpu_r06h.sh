#!/bin/bash
# Round 6: the closed-loop tick at 65,536 robots, eager vs HIP-graph replay, this round's product
# vs round 5's source (the r06z bench line had the graph 26 % behind eager).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_r5 libcmpc; do
  echo "== $v"
  timeout -k 10 300 python -u tools/loop_graph.py 65536 24 $L/$v.so 2>&1 | grep "^B " || exit 1
done
echo done
