#!/bin/bash
# Round 5: no acceptance while a downdated refinement stalls above a tenth of the tolerance --
# GPU tests, parity survey of the product and of the light-bin schedule on top of it, tail
# anatomy, shard rehearsal, A/B against the build before (libcmpc_prev.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -10
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
for v in libcmpc libcmpc_lsd; do
  CMPC_LIB=$L/$v.so timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_gpu_$v.log; exit 1; }
  timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu_$v.log 2>&1 || { tail -5 gpurun_out/survey_cpu_$v.log; exit 1; }
  cp gpurun_out/parity_survey.txt gpurun_out/parity_survey_$v.txt
  echo "== $v"; grep -E "above 1e-4" gpurun_out/survey_cpu_$v.log
done
CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
grep -E "^cfg|max:|8 ranks" gpurun_out/diag_counts.txt
for v in libcmpc libcmpc_lsd; do
  timeout -k 10 300 python -u tools/shard_times.py $L/$v.so 5 > gpurun_out/shard_$v.log 2>&1 || { tail -5 gpurun_out/shard_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/shard_$v.log | grep N=
done
for i in 39503 25651; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 3 > gpurun_out/trace_cfg3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_cfg3_$i.txt; exit 1; }
  tail -2 gpurun_out/trace_cfg3_$i.txt
done
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_prev.so $L/libcmpc_lsd.so || exit 1
echo done
