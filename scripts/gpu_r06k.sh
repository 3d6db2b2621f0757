#!/bin/bash
# Round 6: the closed-loop graph replay at 65,536 robots, bisected on the device code: the product,
# the product without the certified face bound (certified_faces -> true: the spills and scratch of
# round 5, 32 / 76 B per lane), the product with no stats pointer, round 5's source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in ${VARIANTS:-libcmpc libcmpc_nocert libcmpc_nostats libcmpc_r5 libcmpc_nocert}; do
  echo "== $v"
  timeout -k 10 200 python -u tools/loop_graph.py 65536 12 $L/$v.so 2>&1 | grep "^B " || exit 1
done
echo done
