#!/bin/bash
# Round 6: the N = 1/2/4/8 shard rehearsal of config 3 under the runtime settings the r06f sweep
# measured at N = 1 (does any of them shorten the N = 8 straggler tail?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
for p in "" polish_stable=2 polish_repairs=4 polish_repairs=8 alpha=1.4 adaptive_rho_interval=15 adaptive_rho_interval=40 rho=2e-4 ""; do
  CMPC_PARAMS=$p timeout -k 10 200 python -u tools/shard_times.py "" 5 > $O/shard.log 2>&1 || { tail -5 $O/shard.log; exit 1; }
  echo "== ${p:-default}"; grep -E "N=(1|8)" $O/shard.log
done
echo done
