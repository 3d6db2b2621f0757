#!/bin/bash
# Round 5: give up a polish session whose face sets are still far off after 2 / 3 repairs
# (libcmpc_ab2.so / libcmpc_ab3.so) -- A/B against the product, shard rehearsal, parity survey.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_ab2.so $L/libcmpc_ab3.so || exit 1
for v in libcmpc_ab2 libcmpc_ab3; do
  timeout -k 10 300 python -u tools/shard_times.py $L/$v.so 5 > gpurun_out/shard_$v.log 2>&1 || { tail -5 gpurun_out/shard_$v.log; exit 1; }
  echo "== $v"; grep N= gpurun_out/shard_$v.log
done
for v in libcmpc_ab2 libcmpc_ab3; do
  CMPC_LIB=$L/$v.so timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_gpu_$v.log; exit 1; }
  timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_cpu_$v.log; exit 1; }
  cp gpurun_out/parity_survey.txt gpurun_out/parity_survey_$v.txt
  echo "== $v"; grep -E "above 1e-4" gpurun_out/survey_cpu_$v.log | sed 's/.*max/max/'
done
echo done
