#!/bin/bash
# Round 5: the light-bin polish schedule (CMPC_LIGHT_STABLE_DELTA=1, libcmpc_lsd.so) on the LDL'
# product -- GPU tests and the parity survey on it, A/B, shard rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
export CMPC_LIB=$L/libcmpc_lsd.so
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_lsd.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_lsd.log; grep -E "^FAILED" gpurun_out/gpu_tests_lsd.log | head -10
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
timeout -k 10 300 python -u tools/shard_times.py $L/libcmpc_lsd.so 5 > gpurun_out/shard_lsd.log 2>&1 || { tail -5 gpurun_out/shard_lsd.log; exit 1; }
cat gpurun_out/shard_lsd.log
unset CMPC_LIB
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536 1:256" bash scripts/gpu_ab.sh $L/libcmpc_lsd.so $L/libcmpc.so || exit 1
echo done
