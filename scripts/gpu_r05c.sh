#!/bin/bash
# Round 5: GPU tests on the product library (ambiguous-multiplier re-refinement) and on the
# Riccati variant (libcmpc_ric.so, -DCMPC_RICCATI=1), the A/B of both against round 4, the
# parity survey of the product library, traces of the round-5 survey's worst instances.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
CMPC_LIB=$L/libcmpc_ric.so timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_ric.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_ric.log; grep -E "^FAILED" gpurun_out/gpu_tests_ric.log | head -20
case $rc in 124|134|137|139) echo "ric tests aborted ($rc)"; exit 1;; esac
CMPC_ALLOW_ABI4=1 TESTS=0 R=2 CASES="3:65536 2:4096 2:65536 3:8192" bash scripts/gpu_ab.sh $L/libcmpc_r04.so $L/libcmpc.so $L/libcmpc_ric.so || exit 1
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 900 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
for i in 54289 21027; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 3 > gpurun_out/trace_cfg3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_cfg3_$i.txt; exit 1; }
done
echo done
