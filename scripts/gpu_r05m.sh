#!/bin/bash
# Round 5: parity survey + A/B of (a) the narrow stall rule with the LDS-turn apply (the r05h
# build), (b) the acceptance guard with the LDS-turn apply, against the product (guard + register
# turns); warm trace of next-tick instance 17587 on the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 120 python -u tools/trace_instance.py 17587 3 65536 warm > gpurun_out/trace_warm_17587.txt 2>&1 || { tail -5 gpurun_out/trace_warm_17587.txt; exit 1; }
tail -2 gpurun_out/trace_warm_17587.txt
for v in libcmpc_a libcmpc_b; do
  CMPC_LIB=$L/$v.so timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_gpu_$v.log; exit 1; }
  timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_cpu_$v.log; exit 1; }
  cp gpurun_out/parity_survey.txt gpurun_out/parity_survey_$v.txt
  echo "== $v"; grep -E "above 1e-4" gpurun_out/survey_cpu_$v.log | sed 's/.*max/max/'
done
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc_a.so $L/libcmpc_b.so $L/libcmpc.so || exit 1
echo done
