#!/bin/bash
# The round's closing record on one GPU box: GPU tests on the product library, the bench line +
# rocprofv3 + PMC passes (gpu_profile.sh), the one-GPU shard rehearsal, per-phase stamps and the
# per-instance anatomy (tools/summarize_profile.py --tag <tag> then files them under profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit 1; }
bash scripts/gpu_profile.sh || exit 1
timeout -k 10 300 python tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
grep "N=" gpurun_out/shard_rehearsal.log
for c in 1 2; do
  timeout -k 10 120 python tools/stamps.py --config $c --batch 8192 --team 0 --lib $L/libcmpc_stamps.so > gpurun_out/stamps_cfg$c.txt 2>&1 || { tail -5 gpurun_out/stamps_cfg$c.txt; exit 1; }
done
timeout -k 10 120 python tools/stamps.py --config 1 --batch 256 --lib $L/libcmpc_stamps.so > gpurun_out/stamps_team_b256.txt 2>&1 || { tail -5 gpurun_out/stamps_team_b256.txt; exit 1; }
timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
grep -A3 "^cfg3" gpurun_out/diag_counts.txt
echo done
