#!/bin/bash
# Team-mode bring-up: its parity tests alone, then config 1 at B = 256 with the mode on / off
# and a few batch sizes around the automatic threshold.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_team.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/team_test.log 2>&1
rc=$?; tail -15 gpurun_out/team_test.log; [ $rc -eq 0 ] || exit 1
CASES=${CASES:-"1:256 1:512 2:512 2:1024 3:1024"}
for cb in $CASES; do
  cfg=${cb%%:*}; B=${cb##*:}
  for team in 99999 0; do
    timeout -k 10 120 python bench.py --aux 0 --config $cfg --batch $B --steps 50 --team $team > gpurun_out/tb_${cfg}_${B}_$team.json 2> gpurun_out/tb_${cfg}_${B}_$team.err || { echo "bench $cfg $B $team failed"; tail -5 gpurun_out/tb_${cfg}_${B}_$team.err; exit 1; }
    python -c "import json;a=json.load(open('gpurun_out/tb_${cfg}_${B}_$team.json'));print('cfg $cfg B %6d team %5d: %9.0f solves/s %7.3f ms/step ok %.4f itmax %d'%($B,$team,a['value'],a['ms_per_step'],a['solved_frac'],a['iters_max']))"
  done
done
echo done
