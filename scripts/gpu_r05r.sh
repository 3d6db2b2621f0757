#!/bin/bash
# Round 5: which instances a 3-downdate cap stalls (config 2 at 4,096), and a trace of the first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 120 python - <<'PY' > gpurun_out/dd3_fail.txt 2>&1 || { tail -5 gpurun_out/dd3_fail.txt; exit 1; }
import sys, numpy as np
sys.path.insert(0, "convex-mpc-unitree-go2_amd")
from cmpc import _lib
_lib._lib = _lib.load("convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_dd3.so")
from cmpc import Plan, SolverParams, to_device_batch, synth
b = synth.make_config(2, B=4096)
d = to_device_batch(b)
plan = Plan(SolverParams(max_batch=4096))
plan.set_team(0)
w, st, it = plan.solve(*(d[k] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")))
st = st.cpu().numpy(); it = it.cpu().numpy()
bad = np.nonzero(st != 1)[0]
print("failing", len(bad), "first", bad[:10].tolist(), "status", np.unique(st, return_counts=True))
print("IDS", " ".join(map(str, bad[:2])))
PY
cat gpurun_out/dd3_fail.txt
ids=$(grep IDS gpurun_out/dd3_fail.txt | cut -d' ' -f2-)
for i in $ids; do
  timeout -k 10 120 python -u tools/trace_instance.py $i 2 4096 > gpurun_out/trace_dd3_$i.txt 2>&1 || { tail -5 gpurun_out/trace_dd3_$i.txt; exit 1; }
  tail -2 gpurun_out/trace_dd3_$i.txt
done
echo done
