#!/bin/bash
# Round 5: ldl_apply with register-only layout turns (libcmpc_dpp.so) -- GPU tests on it, stamps,
# A/B against the product build without them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
CMPC_LIB=$L/libcmpc_dpp.so timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_dpp.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_dpp.log; grep -E "^FAILED|Error" gpurun_out/gpu_tests_dpp.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/stamps.py --config 2 --batch 8192 --team 0 --lib $L/libcmpc_dpp_stamps.so > gpurun_out/stamps_dpp_cfg2.txt 2>&1 || { tail -5 gpurun_out/stamps_dpp_cfg2.txt; exit 1; }
grep -E "==|per call|instance total|mean iters" gpurun_out/stamps_dpp_cfg2.txt
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc_dpp.so $L/libcmpc.so || exit 1
CMPC_LIB=$L/libcmpc_dpp.so timeout -k 10 300 python -u tools/shard_times.py $L/libcmpc_dpp.so 5 > gpurun_out/shard_dpp.log 2>&1 || { tail -5 gpurun_out/shard_dpp.log; exit 1; }
cat gpurun_out/shard_dpp.log
echo done
