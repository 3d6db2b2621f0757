"""Diagnostic: trace instances INSIDE a full batch, then the same instances alone.

A library built with -DCMPC_TRACE_IDS=i,j,... prints (device printf, every line prefixed "[i]")
the ADMM iterations, polish sessions, refinements, downdates and the final status of those batch
indices.  Inside the batch a wave solves other instances before and after the traced one; alone
(the instance replicated over the whole batch, so its index holds a copy of itself) every wave
only ever sees copies of it.  The first line where the two traces of an instance differ is where
the result starts to depend on the wave's previous instance.
   usage: python tools/trace_batch.py LIB CONFIG B OUTDIR ID [ID ...]   (GPU)"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))

KEYS = ("Ad", "Bd", "gd", "x0", "xref", "contact")


def main():
    lib, cfg, B, outdir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), Path(sys.argv[4])
    ids = [int(x) for x in sys.argv[5:]]
    mode = "batch"
    if ids and ids[0] < 0:  # "-1 ID": the alone run of ID (one process per run: printf order)
        mode, ids = "alone", ids[1:]
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(lib)
    from cmpc import Plan, SolverParams, to_device_batch, synth
    b = synth.make_config(cfg, B=B)
    plan = Plan(SolverParams(max_batch=B))
    plan.set_team(0)
    if mode == "batch":
        d = to_device_batch(b)
        w, st, it = plan.solve(*(d[k] for k in KEYS))
        torch.cuda.synchronize()
        st = st.cpu().numpy()
        it = it.cpu().numpy()
        bad = np.nonzero(st != 1)[0]
        print("BATCH failing", len(bad), "status", dict(zip(*np.unique(st, return_counts=True))),
              flush=True)
        print("TRACED", " ".join(f"{i}:{st[i]}/{it[i]}" for i in ids), flush=True)
    else:
        i = ids[0]
        one = {k: np.repeat(b[k][i:i + 1], B, axis=0) for k in KEYS}
        d = to_device_batch(one)
        w, st, it = plan.solve(*(d[k] for k in KEYS))
        torch.cuda.synchronize()
        print("ALONE", i, int(st.cpu()[i]), int(it.cpu()[i]), flush=True)


if __name__ == "__main__":
    main()
