#!/bin/bash
# instances that do not reach status 1, over the cfg2 A/B seeds (product build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for seed in 11 22 33 44 55; do
  timeout -k 10 120 python tools/find_stuck.py $seed $1 2>/dev/null || exit 1
done
