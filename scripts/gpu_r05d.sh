#!/bin/bash
# Round 5: per-phase stamps and per-instance anatomy of the product library and the Riccati
# variant; A/B of the two (config 3 at 65,536, config 2 at 4,096).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in stamps ric_stamps; do
  for c in 1 2; do
    timeout -k 10 120 python tools/stamps.py --config $c --batch 8192 --team 0 --lib $L/libcmpc_$v.so > gpurun_out/st_${v}_cfg$c.txt 2>&1 || { tail -5 gpurun_out/st_${v}_cfg$c.txt; exit 1; }
    grep -E "==|per call|condense |invert |gradient |symv |instance total|mean iters" gpurun_out/st_${v}_cfg$c.txt
  done
done
for v in diag ric_diag; do
  CMPC_DIAG_LIB=$L/libcmpc_$v.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/dc_$v.txt 2>&1 || { tail -5 gpurun_out/dc_$v.txt; exit 1; }
  grep -E "^cfg|max:|8 ranks" gpurun_out/dc_$v.txt
done
TESTS=0 R=2 CASES="3:65536 2:4096" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_ric.so
