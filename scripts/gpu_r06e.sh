#!/bin/bash
# Round 6: polish_refine 2 as the default (v7): every GPU test; A/B against round 5's product and
# against polish_refine 1 / 4 on this build (config 3 at 65,536, config 2 at 4,096, config 1 at
# 256); the N = 1/2/4/8 shard rehearsal for each setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export CMPC_ALLOW_ABI5=1
O=gpurun_out/r06e; mkdir -p $O
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
BA="--sub-configs 0 --cpu-seconds 0 --aux 0 --steps 20"
for r in 1 2; do
  for cb in 3:65536 2:4096 1:256; do
    for v in "r5:$L/libcmpc_r5.so:" "pr2:$L/libcmpc.so:" "pr1:$L/libcmpc.so:--param polish_refine=1" "pr4:$L/libcmpc.so:--param polish_refine=4"; do
      tag=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; extra=${rest#*:}
      timeout -k 10 300 python bench.py --config ${cb%%:*} --batch ${cb##*:} $BA --lib $lib $extra > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
      python -c "import json;a=json.load(open('$O/ab.json'));print('%-6s %-9s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('$tag','$cb',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
    done
  done
done
for pr in 2 1 4; do
  CMPC_PARAMS=polish_refine=$pr timeout -k 10 300 python -u tools/shard_times.py "" 5 > $O/shard_pr$pr.log 2>&1 || { tail -5 $O/shard_pr$pr.log; exit 1; }
  echo "polish_refine $pr"; grep "N=" $O/shard_pr$pr.log
done
echo done
