#!/bin/bash
# Round 6: at least 4 refinement steps in a warm polish session (libcmpc_warm4): the bench line
# (warm throughput, closed loop) of the product and of it, then every GPU test and the warm
# survey sets (plus config 3 cold) with it as libcmpc.so (this box's copy only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib; O=gpurun_out/r06w; mkdir -p $O
for v in libcmpc libcmpc_warm4; do
  timeout -k 10 400 python bench.py --sub-configs 0 --cpu-seconds 0 --lib $L/$v.so > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python -c "import json;a=json.load(open('$O/bench_$v.json'));w=a['warm_start'];c=a['closed_loop'];print('$v cold %.3f ms, warm %.2f M/s (x%.2f), loop65536 %.3f/%.3f, loop1024 %.3f'%(a['ms_per_step'],w['solves_per_s_warm']/1e6,w['speedup'],c['robots_65536']['ms_per_tick_eager'],c['robots_65536']['ms_per_tick_graph'],c['robots_1024']['ms_per_tick_graph']))"
done
cp $L/libcmpc_warm4.so $L/libcmpc.so
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -10
case $rc in 0|1) ;; *) echo "tests aborted ($rc)"; exit 1;; esac
S=cfg2_next_warm,cfg2_next_ref,cfg3_next_warm,mixed_s13_next_warm,cfg3_65536
SURVEY_DIR=/tmp/svw timeout -k 10 300 python -u tests/certify_sample.py gpu --sets $S > $O/survey_gpu.log 2>&1 || { tail -5 $O/survey_gpu.log; exit 1; }
SURVEY_DIR=/tmp/svw timeout -k 10 600 python -u tests/certify_sample.py cpu --sets $S --report $O/survey.txt > $O/survey_cpu.log 2>&1 || { tail -5 $O/survey_cpu.log; exit 1; }
grep -E "instances|status:|above 1e-4|NOT" $O/survey.txt | cut -c1-170
echo done
