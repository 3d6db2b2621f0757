#!/bin/bash
# Round 5, first call: GPU tests on the new library (float64 rollout in the polish, face
# multipliers in force units, no interior-point variant), the parity survey (every instance of
# eight batches certified on the box's CPU), then an A/B against the round-4 library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
cat gpurun_out/survey_gpu.log
timeout -k 10 1100 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
CMPC_ALLOW_ABI4=1 TESTS=0 R=2 CASES="${CASES:-3:65536 2:4096 1:256}" bash scripts/gpu_ab.sh $L/libcmpc_r04.so $L/libcmpc.so
