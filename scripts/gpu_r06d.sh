#!/bin/bash
# Round 6: the product with the one-step re-check after a stall refactor (v5): every GPU test,
# A/B against round 5's product and this round's first guard build (v4), the minimum polish
# refinement at 2 (runtime parameter), and the parity survey of both settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
O=gpurun_out/r06d; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
export BENCH_ARGS="--sub-configs 0 --cpu-seconds 0"
TESTS=0 R=2 CASES="3:65536 2:4096" bash scripts/gpu_ab.sh $L/libcmpc_r5.so $L/libcmpc_v4.so $L/libcmpc.so 2>&1 | grep -v "^done" || exit 1
for cb in 3:65536 2:4096 3:65536 2:4096; do
  timeout -k 10 300 python bench.py --aux 0 --config ${cb%%:*} --batch ${cb##*:} --steps 20 $BENCH_ARGS --param polish_refine=2 > $O/pr2.json 2> $O/pr2.err || { tail -5 $O/pr2.err; exit 1; }
  python -c "import json;a=json.load(open('$O/pr2.json'));print('%-40s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('polish_refine=2 $cb',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
done
SURVEY_DIR=/tmp/sv1 timeout -k 10 300 python -u tests/certify_sample.py gpu > $O/survey_gpu.log 2>&1 || { tail -5 $O/survey_gpu.log; exit 1; }
SURVEY_DIR=/tmp/sv1 timeout -k 10 700 python -u tests/certify_sample.py cpu --report $O/survey_v5.txt > $O/survey_cpu.log 2>&1 || { tail -5 $O/survey_cpu.log; exit 1; }
grep -E "above 1e-4|not status 1" $O/survey_v5.txt
SURVEY_DIR=/tmp/sv2 timeout -k 10 300 python -u tests/certify_sample.py gpu --param polish_refine=2 > $O/survey2_gpu.log 2>&1 || { tail -5 $O/survey2_gpu.log; exit 1; }
SURVEY_DIR=/tmp/sv2 timeout -k 10 700 python -u tests/certify_sample.py cpu --report $O/survey_v5_pr2.txt > $O/survey2_cpu.log 2>&1 || { tail -5 $O/survey2_cpu.log; exit 1; }
grep -E "above 1e-4|not status 1" $O/survey_v5_pr2.txt
echo done
