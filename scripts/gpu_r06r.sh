#!/bin/bash
# Round 6: a gate on the polish session's start (experiment build libcmpc_gate, CMPC_POL_GATE =
# g > 0: no session from an ADMM point whose primal residual max|x - z| is above g x the force
# scale).  The traced stragglers (r06q) start their failed first sessions at residuals of 2-4 N
# and spend 6-12 refactoring repairs there.  A/B of gate values, then the N = 8 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib; O=gpurun_out/r06r; mkdir -p $O
export BENCH_ARGS="--sub-configs 0 --cpu-seconds 0"
G=$L/libcmpc_gate.so
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536 1:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $G $G@CMPC_POL_GATE=0.05 $G@CMPC_POL_GATE=0.02 $G@CMPC_POL_GATE=0.01 $G@CMPC_POL_GATE=0.005 2>&1 | grep -v "^done" || exit 1
for g in 0 0.05 0.02 0.01 0.005; do
  CMPC_POL_GATE=$g timeout -k 10 200 python -u tools/shard_times.py $G 5 > $O/shard_$g.log 2>&1 || { tail -5 $O/shard_$g.log; exit 1; }
  echo "gate $g $(grep -E 'N=8' $O/shard_$g.log)"
done
echo done
