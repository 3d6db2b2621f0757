#!/bin/bash
# Round 6: where the 3-downdate-cap build's results start to depend on the wave's previous
# instance.  (1) the cap-3 build traced INSIDE config 2 at 4,096 (ten instances that failed there
# in round 5), then each failing traced instance alone: the first differing trace line is the
# leak.  (2) the park-slab-poisoned cap-3 build: status counts, run to run.  (3) last: the
# LDS-poisoned product build (round 5's missing control).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
O=gpurun_out/r06a; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
IDS="260 282 314 328 334 350 352 356 361 372"
timeout -k 10 240 python -u tools/trace_batch.py $L/libcmpc_dd3tr.so 2 4096 $O $IDS > $O/batch.txt 2>&1 || { tail -5 $O/batch.txt; exit 1; }
grep -E "^(BATCH|TRACED)" $O/batch.txt
bad=$(grep "^TRACED" $O/batch.txt | tr ' ' '\n' | grep ":" | grep -v ":1/" | cut -d: -f1 | head -3)
for i in $bad; do
  timeout -k 10 180 python -u tools/trace_batch.py $L/libcmpc_dd3tr.so 2 4096 $O -1 $i > $O/alone_$i.txt 2>&1 || { tail -5 $O/alone_$i.txt; exit 1; }
  grep "^ALONE" $O/alone_$i.txt
done
CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python -u tools/diag_counts.py > $O/diag_counts.txt 2>&1 || { tail -5 $O/diag_counts.txt; exit 1; }
grep -E "^cfg" $O/diag_counts.txt
for v in libcmpc_dd3pp libcmpc_pl; do
  for r in 1 2; do
    timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so $O/det_${v}_$r.npz > $O/det_${v}_$r.log 2>&1 || { echo "$v run $r failed"; tail -30 $O/det_${v}_$r.log; exit 1; }
  done
  echo "== $v"
  python -c "
import numpy as np
a=np.load('$O/det_${v}_1.npz')
for k in ('cfg3','cfg2','cfg3_next_warm'):
    st=a[k+'_st']; print(k, 'not status 1:', int((st!=1).sum()), 'iters max', int(a[k+'_it'].max()))"
  python tools/bitwise_ab.py --compare $O/det_${v}_1.npz $O/det_${v}_2.npz | tail -1
done
rm -f $O/det_*.npz
echo done
