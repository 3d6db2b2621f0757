#!/bin/bash
# A/B on one GPU box: parity tests on the product library, then the headline workloads
# (configs 3, 2 at 4096 and 65536, 1 at 256) with the product library vs a variant, alternating.
#   usage: bash scripts/gpu_ab.sh <variant.so> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${1:?variant library}
R=${2:-2}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1
  rc=$?; tail -1 gpurun_out/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test.log | head -20; exit 1; }
fi
run() {  # lib cfg batch
  local extra=""; [ "$1" != "base" ] || extra="--lib convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_base.so"
  [ "$1" = "var" ] && extra="--lib $VAR"
  timeout -k 10 300 python bench.py --aux 0 --config $2 --batch $3 --steps ${STEPS:-20} $extra > gpurun_out/ab_$1_$2_$3.json 2> gpurun_out/ab_$1_$2_$3.err || { echo "bench $1 $2 $3 failed"; tail -5 gpurun_out/ab_$1_$2_$3.err; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/ab_$1_$2_$3.json'));print('$1 cfg$2 B=$3 %.0f solves/s %.3f ms/step ok %.5f itmax %d'%(a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
}
for r in $(seq $R); do
  for cb in "3 65536" "2 65536" "2 4096" "1 256" "1 65536"; do
    set -- $cb
    run ${A:-base} $1 $2 || exit 1
    run var $1 $2 || exit 1
  done
done
echo done
