#!/bin/bash
# Round 5: where the 3-downdate-cap build's state leak lives -- NaN poisoning of the wave's LDS
# float scratch (dd3pl) or of its park slab (dd3pp) before every instance; the product build with
# the LDS poisoning (pl) as the control.  Run-to-run determinism and status counts of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc_dd3 libcmpc_dd3pl libcmpc_dd3pp libcmpc_pl; do
  for r in 1 2; do
    timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so gpurun_out/det_${v}_$r.npz > gpurun_out/det_${v}_$r.log 2>&1 || { tail -5 gpurun_out/det_${v}_$r.log; exit 1; }
  done
  echo "== $v"
  python -c "
import numpy as np
a=np.load('gpurun_out/det_${v}_1.npz')
for k in ('cfg3','cfg2','cfg3_next_warm'):
    st=a[k+'_st']; print(k, 'not status 1:', int((st!=1).sum()), 'iters max', int(a[k+'_it'].max()))"
  python tools/bitwise_ab.py --compare gpurun_out/det_${v}_1.npz gpurun_out/det_${v}_2.npz | tail -1
done
rm -f gpurun_out/det_*.npz
echo done
