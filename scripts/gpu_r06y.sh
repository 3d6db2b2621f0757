#!/bin/bash
# Round 6 final record of the product after the plan-stream stats fix (device code bit-identical
# to r06z): every GPU test, smoke, the default bench line + rocprofv3 kernel trace + PMC passes
# (scripts/gpu_profile.sh), the N = 1/2/4/8 shard rehearsal, the closed loop eager vs graph at
# 65,536 and 1,024 robots.  Only libcmpc.so (built by build()) is in the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ls convex-mpc-unitree-go2_amd/cmpc/lib/
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -10
case $rc in 0|1) ;; *) echo "tests aborted ($rc)"; exit 1;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
FULL=1 bash scripts/gpu_profile.sh > gpurun_out/profile_run.log 2>&1 || { tail -5 gpurun_out/profile_run.log; exit 1; }
python -c "import json;a=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1]);c=a['closed_loop'];print('value %.0f ms %.3f roofline %.4f acceptance %s loop65536 eager %.3f graph %.3f loop1024 graph %.3f'%(a['value'],a['ms_per_step'],a['roofline']['frac'],a['acceptance_per_step'],c['robots_65536']['ms_per_tick_eager'],c['robots_65536']['ms_per_tick_graph'],c['robots_1024']['ms_per_tick_graph']))"
timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
grep N= gpurun_out/shard_rehearsal.log
for B in 65536 1024; do
  timeout -k 10 200 python -u tools/loop_graph.py $B 24 > gpurun_out/loop_$B.log 2>&1 || { tail -5 gpurun_out/loop_$B.log; exit 1; }
  grep "^B " gpurun_out/loop_$B.log
done
echo done
