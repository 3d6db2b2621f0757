#!/bin/bash
# Round 6: compiler scheduling strategies for the same source (libcmpc_ilp: max-ilp,
# libcmpc_trk: AMDGPU register-pressure trackers, libcmpc_mclause: max-memory-clause): bitwise
# identity of the outputs against the product, then an A/B of the headline workloads and the
# 257-1,024 team range, and the N = 8 shard rehearsal of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib; O=gpurun_out/r06o; mkdir -p $O
for v in libcmpc libcmpc_ilp libcmpc_trk libcmpc_mclause; do
  timeout -k 10 200 python tools/bitwise_ab.py $L/$v.so $O/$v.npz > $O/bw_$v.log 2>&1 || { tail -5 $O/bw_$v.log; exit 1; }
done
for v in libcmpc_ilp libcmpc_trk libcmpc_mclause; do
  echo "bitwise $v: $(python tools/bitwise_ab.py --compare $O/libcmpc.npz $O/$v.npz 2>&1 | tail -1)"
done
export BENCH_ARGS="--sub-configs 0 --cpu-seconds 0"
TESTS=0 R=2 CASES="3:65536 2:4096 2:1024 1:256" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_ilp.so $L/libcmpc_trk.so $L/libcmpc_mclause.so 2>&1 | grep -v "^done" || exit 1
for v in libcmpc libcmpc_ilp libcmpc_trk libcmpc_mclause; do
  timeout -k 10 200 python -u tools/shard_times.py $L/$v.so 5 > $O/shard_$v.log 2>&1 || { tail -5 $O/shard_$v.log; exit 1; }
  echo "$v $(grep -E 'N=8' $O/shard_$v.log)"
done
echo done
