#!/bin/bash
# Round 5: refactor instead of trusting a stalled downdated refinement -- GPU tests, tail
# anatomy, trace of 31861, shard rehearsal, A/B against the build before (libcmpc_prev.so),
# parity survey.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -20
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
CMPC_DIAG_SAVE=gpurun_out/dg CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
grep -E "^cfg|max:|8 ranks" gpurun_out/diag_counts.txt
ids=$(python -c "import numpy as np; c=np.load('gpurun_out/dg_cfg3.npz')['cyc']; print(' '.join(map(str, np.argsort(c)[::-1][:3])))")
echo "slowest cfg3: $ids"
for i in 31861 $ids; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 3 > gpurun_out/trace_cfg3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_cfg3_$i.txt; exit 1; }
  tail -1 gpurun_out/trace_cfg3_$i.txt
done
timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
cat gpurun_out/shard_rehearsal.log
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_prev.so || exit 1
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
echo done
