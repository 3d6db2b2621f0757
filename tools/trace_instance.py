"""Diagnostic: trace one instance of a benchmark batch through the solver (libcmpc_trace.so,
built with -DCMPC_TRACE=0: device printf of ADMM iterations, polish sessions and the
interior-point steps of batch element 0).  The instance is replicated to 2,048 copies so the
one-wave-per-QP kernels run it (small batches take the team kernel).
   usage: python tools/trace_instance.py INDEX [CONFIG [BATCH]]   (default config 3, 65,536)"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_trace.so")
    from cmpc import Plan, SolverParams, to_device_batch, synth
    i = int(sys.argv[1])
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    b = synth.make_config(cfg, B=B)
    one = {k: np.repeat(b[k][i:i + 1], 2048, axis=0) for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}
    d = to_device_batch(one)
    plan = Plan(SolverParams(max_batch=4096))
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()
    print("status", int(st[0]), "iters", int(it[0]), flush=True)


if __name__ == "__main__":
    main()
