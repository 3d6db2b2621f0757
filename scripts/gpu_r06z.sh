#!/bin/bash
# Round 6 final record on one GPU box: GPU tests, smoke, the default bench line + rocprofv3
# kernel trace + PMC passes (scripts/gpu_profile.sh), a kernel trace of config 1 at 65,536 (the
# NC 192 kernel with an empty bin), N = 1/2/4/8 shard rehearsal, per-instance anatomy, per-phase
# stamps, the parity survey.  tools/summarize_profile.py --tag r06z turns it into profiles/.
# The diagnostic libraries (libcmpc_diag.so, libcmpc_stamps.so) are copied in for this call only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -10
case $rc in 0|1) ;; *) echo "tests aborted ($rc)"; exit 1;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
FULL=1 bash scripts/gpu_profile.sh > gpurun_out/profile_run.log 2>&1 || { tail -5 gpurun_out/profile_run.log; exit 1; }
python -c "import json;a=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1]);print('value %.0f ms %.3f roofline %.4f acceptance %s'%(a['value'],a['ms_per_step'],a['roofline']['frac'],a['acceptance_per_step']))"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_cfg1 -o run --output-format csv -- python bench.py --aux 0 --config 1 --batch 65536 --sub-configs 0 --cpu-seconds 0 --steps 5 --warmup 1 > gpurun_out/prof_cfg1.log 2>&1 || { tail -5 gpurun_out/prof_cfg1.log; exit 1; }
timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
grep N= gpurun_out/shard_rehearsal.log
CMPC_DIAG_SAVE=gpurun_out/diag CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
grep -E "^cfg|max:|8 ranks" gpurun_out/diag_counts.txt
for c in 1 2; do
  timeout -k 10 120 python tools/stamps.py --config $c --batch 8192 --team 0 --lib $L/libcmpc_stamps.so > gpurun_out/stamps_cfg$c.txt 2>&1 || { tail -5 gpurun_out/stamps_cfg$c.txt; exit 1; }
done
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 700 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4" gpurun_out/parity_survey.txt
echo done
