#!/bin/bash
# Round 5: the gradient's per-step params in chunks of 4 (libcmpc_gch.so) -- bit-identity against
# the product, GPU tests on it, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_gch; do
  timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so gpurun_out/bw_$v.npz > gpurun_out/bw_$v.log 2>&1 || { tail -5 gpurun_out/bw_$v.log; exit 1; }
done
python tools/bitwise_ab.py --compare gpurun_out/bw_libcmpc_gch.npz gpurun_out/bw_libcmpc.npz | tee gpurun_out/bitwise_gch.txt
rm -f gpurun_out/bw_*.npz
CMPC_LIB=$L/libcmpc_gch.so timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_gch.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_gch.log; grep -E "^FAILED" gpurun_out/gpu_tests_gch.log | head -10
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
TESTS=0 R=3 CASES="3:65536 2:4096 1:65536" bash scripts/gpu_ab.sh $L/libcmpc_gch.so $L/libcmpc.so || exit 1
echo done
