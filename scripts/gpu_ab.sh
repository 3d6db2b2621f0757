#!/bin/bash
# A/B on one GPU box: (optional) parity tests on the product library, then the headline
# workloads with each given variant, alternating, R rounds.  A variant is a library build,
# optionally with environment settings: path.so[@VAR=val[,VAR=val...]]
#   usage: [TESTS=0] [R=2] [CASES="3:65536 2:4096"] bash scripts/gpu_ab.sh a.so b.so@CMPC_X=1 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
  rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
fi
CASES=${CASES:-"3:65536 2:65536 2:4096 1:256 1:65536"}
for r in $(seq ${R:-2}); do
  for cb in $CASES; do
    cfg=${cb%%:*}; B=${cb##*:}
    for var in "$@"; do
      lib=${var%%@*}; envs=""; [ "$var" != "$lib" ] && envs=${var#*@}
      tag=$(basename $lib .so)$(echo "$envs" | tr -c 'A-Za-z0-9\n' '_' | sed 's/^./_&/')_${cfg}_${B}
      env ${envs//,/ } timeout -k 10 300 python bench.py --aux 0 --config $cfg --batch $B --steps ${STEPS:-20} --lib $lib ${BENCH_ARGS} > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
      python -c "import json;a=json.load(open('gpurun_out/ab_$tag.json'));print('%-40s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('$tag',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
    done
  done
done
echo done
