#!/bin/bash
# Round 5: trace the survey's worst config-3 instances, survey the round-4 library on the same
# batches for comparison, re-survey this build, then the warm-restart / team-occupancy /
# NC 192 grid A/Bs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
for i in ${TRACE_IDS:-54289 21027 52595}; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 3 > gpurun_out/trace_cfg3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_cfg3_$i.txt; exit 1; }
done
SETS=${SETS:-cfg3_65536,cfg3_next_warm,cfg2_next_cold}
CMPC_LIB=$L/libcmpc_r04.so CMPC_ALLOW_ABI4=1 SURVEY_DIR=/tmp/sv_r04 timeout -k 10 300 python -u tests/certify_sample.py gpu --sets $SETS > gpurun_out/survey_r04_gpu.log 2>&1 || { tail -5 gpurun_out/survey_r04_gpu.log; exit 1; }
SURVEY_DIR=/tmp/sv_r04 timeout -k 10 900 python -u tests/certify_sample.py cpu --sets $SETS --report gpurun_out/r04lib/parity_survey.txt > gpurun_out/survey_r04_cpu.log 2>&1 || { tail -5 gpurun_out/survey_r04_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_r04_cpu.log
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 900 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg|status" gpurun_out/survey_cpu.log
W="--cpu-seconds 0 --sub-configs 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 --steps 5"
for v in "$L/libcmpc_r04.so" "$L/libcmpc.so" "$L/libcmpc.so@CMPC_TOP_GRID=64"; do
  lib=${v%%@*}; envs=""; [ "$v" != "$lib" ] && envs=${v#*@}
  env CMPC_ALLOW_ABI4=1 $envs timeout -k 10 300 python bench.py $W --lib $lib > gpurun_out/warm_$(basename $lib .so)${envs:+_top}.json 2>/dev/null || { echo "bench failed $v"; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/warm_$(basename $lib .so)${envs:+_top}.json'));w=a['warm_start'];print('$v', round(a['ms_per_step'],3), 'warm', {k:w[k] for k in ('iters_max_warm','iters_max_cold','iters_mean_warm','solves_per_s_warm','solves_per_s_cold','solved_frac_warm')})"
done
CMPC_ALLOW_ABI4=1 TESTS=0 R=2 CASES="1:1024 2:1024 3:1024" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc.so@CMPC_TEAM_OCC=1
CMPC_ALLOW_ABI4=1 TESTS=0 R=2 CASES="3:65536 2:65536 3:8192" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc.so@CMPC_TOP_GRID=64
