#!/bin/bash
# Round 5: the config-3 tail under the LDL' product -- per-instance anatomy saved, the three
# slowest instances traced (device printf build), then the round's profile (rocprofv3 kernel
# trace + PMC passes, scripts/gpu_profile.sh without the bench line).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
CMPC_DIAG_SAVE=gpurun_out/dg CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
ids=$(python -c "import numpy as np; c=np.load('gpurun_out/dg_cfg3.npz')['cyc']; print(' '.join(map(str, np.argsort(c)[::-1][:3])))")
echo "slowest cfg3: $ids"
for i in $ids; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 3 > gpurun_out/trace_cfg3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_cfg3_$i.txt; exit 1; }
  tail -2 gpurun_out/trace_cfg3_$i.txt
done
FULL=0 bash scripts/gpu_profile.sh || exit 1
echo done
