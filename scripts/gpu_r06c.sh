#!/bin/bash
# Round 6: the product library of this round's source -- every GPU test (not stopping at the
# first failure), bit-identity against the guard-on build measured in r06b, the straggler team
# speed, round 5's cap-3 source without -amdgpu-mfma-vgpr-form (determinism), one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
O=gpurun_out/r06c; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; grep -E "^FAILED|Error" $O/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
for v in libcmpc libcmpc_prodg; do
  timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so $O/bw_$v.npz > $O/bw_$v.log 2>&1 || { tail -5 $O/bw_$v.log; exit 1; }
done
python tools/bitwise_ab.py --compare $O/bw_libcmpc.npz $O/bw_libcmpc_prodg.npz
for r in 1 2; do
  timeout -k 10 300 python -u tools/bitwise_ab.py $L/libcmpc_old_dd3nv.so $O/nv_$r.npz > $O/nv_$r.log 2>&1 || { tail -5 $O/nv_$r.log; exit 1; }
done
echo "== old source, cap 3, without -amdgpu-mfma-vgpr-form"
python tools/bitwise_ab.py --compare $O/nv_1.npz $O/nv_2.npz | tail -1
rm -f $O/*.npz
timeout -k 10 300 python -u tools/straggler_speed.py profiles/r06b_diag/diag_cfg3.npz 8 > $O/straggler_speed.txt 2>&1 || { tail -5 $O/straggler_speed.txt; exit 1; }
cat $O/straggler_speed.txt
TESTS=0 R=2 CASES="3:65536 2:4096" bash scripts/gpu_ab.sh $L/libcmpc_r5.so $L/libcmpc_prodg.so $L/libcmpc.so 2>&1 | grep -v "^done" || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "
import json; a=json.load(open('$O/bench.json'))
print('bench', a['value'], a['ms_per_step'], a['status_counts'], a['acceptance_per_step'], a['roofline']['frac'])
print('shard', a.get('shard_rehearsal'))"
echo done
