#!/bin/bash
# Round 5: run-to-run determinism of the product and of the 3-downdate-cap build (instances meet
# different wave neighbours from run to run: a difference means state leaking between them)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
for v in libcmpc libcmpc_dd3; do
  for r in 1 2; do
    timeout -k 10 300 python -u tools/bitwise_ab.py $L/$v.so gpurun_out/det_${v}_$r.npz > gpurun_out/det_${v}_$r.log 2>&1 || { tail -5 gpurun_out/det_${v}_$r.log; exit 1; }
  done
  echo "== $v run 1 vs run 2"
  python tools/bitwise_ab.py --compare gpurun_out/det_${v}_1.npz gpurun_out/det_${v}_2.npz
done
rm -f gpurun_out/det_*.npz
echo done
