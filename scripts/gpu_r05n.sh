#!/bin/bash
# Round 5: the register-turn apply with the LDS build's arithmetic (mode 2, libcmpc.so) against
# the LDS build (libcmpc_m0.so): bit-identity on three batches, GPU tests, A/B, shard rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_m0; do
  timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so gpurun_out/bw_$v.npz > gpurun_out/bw_$v.log 2>&1 || { tail -5 gpurun_out/bw_$v.log; exit 1; }
done
python tools/bitwise_ab.py --compare gpurun_out/bw_libcmpc.npz gpurun_out/bw_libcmpc_m0.npz | tee gpurun_out/bitwise.txt
rm -f gpurun_out/bw_*.npz
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -10
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
TESTS=0 R=3 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_m0.so || exit 1
timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
grep N= gpurun_out/shard_rehearsal.log
echo done
