#!/bin/bash
# Diagnostic: per-phase stamps at 1 and 2 blocks/CU (libcmpc_stamps.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for bpc in 1 2; do
  CMPC_BLOCKS_PER_CU=$bpc timeout -k 10 300 python tools/stamps.py --config 1 > gpurun_out/occ_$bpc.txt 2>&1 || { cat gpurun_out/occ_$bpc.txt; exit 1; }
  echo "== blocks/CU $bpc"; grep -v amdgpu.ids gpurun_out/occ_$bpc.txt
done
