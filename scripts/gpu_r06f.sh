#!/bin/bash
# Round 6: re-sweep of the runtime solver settings on the LDL' + guard + polish_refine 2 build
# (config 3 at 65,536 and config 2 at 4,096, two alternations each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
BA="--sub-configs 0 --cpu-seconds 0 --aux 0 --steps 20"
for r in 1 2; do
  for cb in 3:65536 2:4096; do
    for p in "" polish_stable=2 polish_stable=4 polish_repairs=4 polish_repairs=8 alpha=1.8 alpha=1.4 adaptive_rho_interval=15 adaptive_rho_interval=40 rho=2e-4 rho=5e-5; do
      extra=""; [ -n "$p" ] && extra="--param $p"
      timeout -k 10 300 python bench.py --config ${cb%%:*} --batch ${cb##*:} $BA $extra > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
      python -c "import json;a=json.load(open('$O/ab.json'));print('%-26s %-9s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('${p:-default}','$cb',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
    done
  done
done
echo done
