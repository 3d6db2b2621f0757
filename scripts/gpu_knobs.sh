#!/bin/bash
# A/B of runtime knobs (no rebuild) on one GPU box: every case with every argument set,
# alternating, R rounds.
#   usage: [R=2] [CASES="3:8192 3:16384"] bash scripts/gpu_knobs.sh "<args A>" "<args B>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASES=${CASES:-"3:65536 3:16384 3:8192 2:4096"}
for r in $(seq ${R:-2}); do
  for cb in $CASES; do
    cfg=${cb%%:*}; B=${cb##*:}
    v=0
    for va in "$@"; do
      v=$((v+1))
      tag=k${v}_${cfg}_${B}
      timeout -k 10 300 python bench.py --aux 0 --sub-configs 0 --config $cfg --batch $B --steps ${STEPS:-20} $va > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/$tag.err; exit 1; }
      python -c "import json;a=json.load(open('gpurun_out/$tag.json'));print('%-14s %-28s %9.0f solves/s %7.3f ms/step ok %.5f itmax %d'%('$tag','$va',a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
    done
  done
done
echo done
