#!/bin/bash
# Round 6: the one-workgroup-per-CU team image (<4,1>, 0 spills, persistent over B / CUs
# instances per workgroup; CMPC_TEAM_OCC=1) against the two-per-CU image (<4,2>, 157 spills) on
# CUs < B <= 4 x CUs, configs 1-3, and the 1,024-robot closed loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
BA="--sub-configs 0 --cpu-seconds 0 --aux 0 --steps 50"
for r in 1 2; do
  for cb in 1:512 1:1024 2:512 2:1024 3:512 3:1024; do
    for occ in 0 1; do
      CMPC_TEAM_OCC=$occ timeout -k 10 200 python bench.py --config ${cb%%:*} --batch ${cb##*:} $BA > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
      python -c "import json;a=json.load(open('$O/ab.json'));print('occ %s %-7s %8.4f ms/step ok %.5f itmax %d %s'%('$occ','$cb',a['ms_per_step'],a['solved_frac'],a['iters_max'],a['roofline'].get('kernel')))"
    done
  done
done
for occ in 0 1 0 1; do
  echo "closed loop 1024 occ $occ"
  CMPC_TEAM_OCC=$occ timeout -k 10 200 python -u tools/loop_graph.py 1024 48 "" eager,graph 2>&1 | grep "^B " || exit 1
done
echo done
