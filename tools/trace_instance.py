"""Diagnostic: trace one instance of a benchmark batch through the solver (libcmpc_trace.so,
built with -DCMPC_TRACE=0: device printf of ADMM iterations, polish sessions and the
interior-point steps of batch element 0).  The instance is replicated to 2,048 copies so the
one-wave-per-QP kernels run it (small batches take the team kernel).
   usage: python tools/trace_instance.py INDEX [CONFIG [BATCH [warm]]]   (default config 3, 65,536;
   warm: then the next tick's solve warm-started from it, as tests/certify_sample.py's *_next_warm)"""
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
    warm = len(sys.argv) > 4 and sys.argv[4] == "warm"
    b = synth.make_config(cfg, B=B)
    keys = ("Ad", "Bd", "gd", "x0", "xref", "contact")
    one = {k: np.repeat(b[k][i:i + 1], 2048, axis=0) for k in keys}
    d = to_device_batch(one)
    plan = Plan(SolverParams(max_batch=4096))
    y = torch.empty((2048, 12 * 16), dtype=torch.float32, device=d["Ad"].device)
    w, st, it = plan.solve(*(d[k] for k in keys), y_out=y)
    torch.cuda.synchronize()
    print("status", int(st[0]), "iters", int(it[0]), flush=True)
    if warm:  # the next tick (synth.next_tick of the whole batch), warm from this (w, y)
        nt = synth.next_tick(b)
        d2 = to_device_batch({k: np.repeat(nt[k][i:i + 1], 2048, axis=0) for k in keys})
        print("---- next tick, warm", flush=True)
        w2, st2, it2 = plan.solve(*(d2[k] for k in keys), w_init=w, y_init=y)
        torch.cuda.synchronize()
        print("status", int(st2[0]), "iters", int(it2[0]), flush=True)


if __name__ == "__main__":
    main()
