#!/bin/bash
# Round 6: the refinement error bound in the status-1 contract (libcmpc_refb): a polished point
# whose last refinement step contracted by r > 1/2 is status 1 only if step x r / (1 - r) <=
# 4e-5 x the force scale (a fresh-seed warm tick held two status-1 answers at 1.1e-4 and 2.1e-4).
# A/B against the product, then every GPU test and the whole parity survey (the eight standard
# sets and the three fresh-seed sets) with it as libcmpc.so (this box's copy only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib; O=gpurun_out/r06s; mkdir -p $O
export BENCH_ARGS="--sub-configs 0 --cpu-seconds 0"
TESTS=0 R=2 CASES="3:65536 2:4096 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_refb.so 2>&1 | grep -v "^done" || exit 1
for v in libcmpc libcmpc_refb; do
  python -c "import json;a=json.load(open('gpurun_out/ab_${v}_3_65536.json'));print('$v', a['status_counts'], a['acceptance_per_step'])"
done
cp $L/libcmpc_refb.so $L/libcmpc.so
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -10
case $rc in 0|1) ;; *) echo "tests aborted ($rc)"; exit 1;; esac
S=cfg2_next_cold,cfg2_next_warm,cfg2_next_ref,cfg2_4096,cfg1_256,cfg3_65536,cfg3_next_warm,cfg2_65536,mixed_s11_65536,trot_s12_65536,mixed_s13_next_warm
SURVEY_DIR=/tmp/svs timeout -k 10 400 python -u tests/certify_sample.py gpu --sets $S > $O/survey_gpu.log 2>&1 || { tail -5 $O/survey_gpu.log; exit 1; }
SURVEY_DIR=/tmp/svs timeout -k 10 900 python -u tests/certify_sample.py cpu --sets $S --report $O/survey.txt > $O/survey_cpu.log 2>&1 || { tail -5 $O/survey_cpu.log; exit 1; }
grep -E "instances|status:|above 1e-4|NOT" $O/survey.txt
echo done
