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
# small batches: the team kernel's two-per-CU image (B 257..1,024) vs the one-wave kernels
for cb in 2:512 2:1024 3:1024 1:1024; do
  cfg=${cb%%:*}; B=${cb##*:}
  for t in -1 256; do
    timeout -k 10 120 python bench.py --aux 0 --config $cfg --batch $B --steps 20 --team $t > gpurun_out/tm_${cfg}_${B}_$t.json 2> gpurun_out/tm.err || { tail -5 gpurun_out/tm.err; exit 1; }
    python -c "import json;a=json.load(open('gpurun_out/tm_${cfg}_${B}_$t.json'));print('cfg $cfg B $B team $t: %.3f ms itmax %d'%(a['ms_per_step'],a['iters_max']))"
  done
done
LOOP="--sub-configs 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --api-ticks 0 --warm-steps 0 --cpu-seconds 1"
for t in -1 256; do
  timeout -k 10 300 python bench.py $LOOP --team $t > gpurun_out/loop_$t.json 2> gpurun_out/loop.err || { tail -5 gpurun_out/loop.err; exit 1; }
  python -c "import json;a=json.loads(open('gpurun_out/loop_$t.json').read().strip().splitlines()[-1]);c=a['closed_loop']['robots_1024'];print('loop 1024 team $t: graph %.3f ms eager %.3f ms'%(c['ms_per_tick_graph'],c['ms_per_tick_eager']))"
done
echo done
