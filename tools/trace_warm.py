"""Diagnostic: trace instances of a warm next tick (a -DCMPC_TRACE_IDS build prints the ADMM
iterations, polish sessions, refinements, repairs and the final status of those indices).
The previous tick is solved cold first (its trace lines come before the "== warm" marker), then
the next tick (synth.next_tick) warm from its (w, y_out).
   usage: python tools/trace_warm.py LIB SEED [mixed=1] [ID,ID,...: save their rows]   (GPU)"""
import functools
import sys
from pathlib import Path

import numpy as np

print = functools.partial(print, flush=True)
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(sys.argv[1])
    from cmpc import Plan, SolverParams, to_device_batch, synth
    seed = int(sys.argv[2])
    mixed = len(sys.argv) < 4 or sys.argv[3] == "1"
    prev = synth.make_batch(65536, seed, mixed=mixed)
    nxt = synth.next_tick(prev)
    plan = Plan(SolverParams(max_batch=65536))
    p, d = to_device_batch(prev), to_device_batch(nxt)
    print("== cold (previous tick)")
    w0, _, _, y0 = plan.solve(p["Ad"], p["Bd"], p["gd"], p["x0"], p["xref"], p["contact"], y_out=True)
    torch.cuda.synchronize()
    print("== warm")
    w, st, it, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                              w_init=w0, y_init=y0, y_out=True)
    torch.cuda.synchronize()
    print("== done", np.unique(st.cpu().numpy(), return_counts=True))
    ids = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else []
    if ids:  # the warm answers of these instances (and their previous-tick answers)
        np.savez(REPO / "gpurun_out" / "trace_warm_rows.npz", ids=np.array(ids),
                 w=w[ids].cpu().numpy(), st=st[ids].cpu().numpy(), w_prev=w0[ids].cpu().numpy())


if __name__ == "__main__":
    main()
