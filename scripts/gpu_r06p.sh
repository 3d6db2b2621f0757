#!/bin/bash
# Round 6: a repair that frees faces added since the polish factorization rebuilds the face
# downdates from the basis's face set instead of refactoring (libcmpc_rebuild).  A/B against the
# product on the headline workloads and the N = 8 shard rehearsal, then every GPU test and the
# parity survey with it as libcmpc.so (this box's copy only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib; O=gpurun_out/r06p; mkdir -p $O
export BENCH_ARGS="--sub-configs 0 --cpu-seconds 0"
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536 1:256 2:1024" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_rebuild.so 2>&1 | grep -v "^done" || exit 1
for v in libcmpc libcmpc_rebuild; do
  timeout -k 10 200 python -u tools/shard_times.py $L/$v.so 5 > $O/shard_$v.log 2>&1 || { tail -5 $O/shard_$v.log; exit 1; }
  echo "$v $(grep -E 'N=8' $O/shard_$v.log)"
done
cp $L/libcmpc_rebuild.so $L/libcmpc.so
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -10
case $rc in 0|1) ;; *) echo "tests aborted ($rc)"; exit 1;; esac
SURVEY_DIR=/tmp/svr timeout -k 10 300 python -u tests/certify_sample.py gpu > $O/survey_gpu.log 2>&1 || { tail -5 $O/survey_gpu.log; exit 1; }
SURVEY_DIR=/tmp/svr timeout -k 10 700 python -u tests/certify_sample.py cpu --report $O/survey.txt > $O/survey_cpu.log 2>&1 || { tail -5 $O/survey_cpu.log; exit 1; }
grep -E "above 1e-4|not status 1" $O/survey.txt
echo done
