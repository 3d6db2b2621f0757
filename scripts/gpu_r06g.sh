#!/bin/bash
# Round 6: candidate changes on top of the product (v7 = libcmpc.so): modified Gram-Schmidt in
# the face downdates (mgs: one pass, mgs2: two), the light-bin polish schedule (NC <= 128 bins
# polish one stable iteration earlier).  Per-instance anatomy of v7 and mgs (stall re-checks),
# A/B, shard rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in diag7 diagmgs; do
  CMPC_DIAG_LIB=$L/libcmpc_$v.so timeout -k 10 300 python tools/diag_counts.py > $O/diag_$v.txt 2>&1 || { tail -5 $O/diag_$v.txt; exit 1; }
  echo "== $v"; grep -E "^cfg" $O/diag_$v.txt
done
BA="--sub-configs 0 --cpu-seconds 0 --aux 0 --steps 20"
for r in 1 2; do
  for cb in 3:65536 2:4096 2:65536; do
    for v in libcmpc libcmpc_mgs libcmpc_mgs2 libcmpc_light; do
      timeout -k 10 300 python bench.py --config ${cb%%:*} --batch ${cb##*:} $BA --lib $L/$v.so > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
      python -c "import json;a=json.load(open('$O/ab.json'));print('%-16s %-9s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('$v','$cb',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
    done
  done
done
for v in libcmpc_mgs libcmpc_light; do
  timeout -k 10 300 python -u tools/shard_times.py $L/$v.so 5 > $O/shard_$v.log 2>&1 || { tail -5 $O/shard_$v.log; exit 1; }
  echo "== $v"; grep "N=" $O/shard_$v.log
done
echo done
