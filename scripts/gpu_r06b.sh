#!/bin/bash
# Round 6: (1) run-to-run determinism of the 3-downdate-cap build from this round's source and
# from round 5's committed source (round 5 recorded its cap-3 binary as non-deterministic);
# (2) the guard-on product: per-instance anatomy (diag counts, saved for the two-phase model),
# A/B against round 5's product, shard rehearsal; (3) last, the LDS-poisoned cap-3 builds (round
# 5's faulting configuration): this round's source, then round 5's.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
O=gpurun_out/r06b; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
det() {
  v=$1
  for r in 1 2; do
    timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so $O/det_${v}_$r.npz > $O/det_${v}_$r.log 2>&1 || { echo "$v run $r failed"; tail -30 $O/det_${v}_$r.log; return 1; }
  done
  echo "== $v"
  python -c "
import numpy as np
a=np.load('$O/det_${v}_1.npz')
for k in ('cfg3','cfg2','cfg3_next_warm'):
    st=a[k+'_st']; print(k, 'status', dict(zip(*[x.tolist() for x in np.unique(st, return_counts=True)])), 'iters max', int(a[k+'_it'].max()))"
  python tools/bitwise_ab.py --compare $O/det_${v}_1.npz $O/det_${v}_2.npz | tail -1
  rm -f $O/det_${v}_*.npz
}
det libcmpc_new_dd3 || exit 1
det libcmpc_old_dd3 || exit 1
CMPC_DIAG_SAVE=$O/diag CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python -u tools/diag_counts.py > $O/diag_counts.txt 2>&1 || { tail -5 $O/diag_counts.txt; exit 1; }
grep -E "^cfg" $O/diag_counts.txt
TESTS=0 R=2 CASES="3:65536 2:4096 1:256" bash scripts/gpu_ab.sh $L/libcmpc_r5.so $L/libcmpc_prodg.so 2>&1 | grep -v "^done" || exit 1
timeout -k 10 300 python -u tools/shard_times.py $L/libcmpc_prodg.so 3 > $O/shard_prodg.log 2>&1 || { tail -5 $O/shard_prodg.log; exit 1; }
tail -4 $O/shard_prodg.log
det libcmpc_new_dd3pl || exit 1
det libcmpc_old_dd3pl || exit 1
echo done
