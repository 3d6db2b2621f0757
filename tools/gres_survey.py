"""Diagnostic (round 6): per instance of a set, the certified error against the KKT-certified
optimum and the accepted point's own error metrics from a -DCMPC_DIAG_GRES build (w[0] = |grad|_2
at the final refinement point, w[1] = |c|_2, both / (min 2R x force scale); w[2] = the force
scale).  GPU phase solves and saves; the CPU phase certifies every instance (16 processes) and
writes a small npz (err, gm, cm, us, status, iters).
    python tools/gres_survey.py LIB SET OUT.npz        (GPU box: both phases)"""
import sys
import time
from multiprocessing import get_context
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tests"), str(REPO), str(REPO / "convex-mpc-unitree-go2_amd")]


def main():
    lib, name, out = sys.argv[1], sys.argv[2], Path(sys.argv[3])
    import certify_sample as cs
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(lib)
    from cmpc import Plan, SolverParams, to_device_batch
    b, prev = cs.batch_of(name)
    plan = Plan(SolverParams(max_batch=65536))
    d = to_device_batch(b)
    if prev is None:
        w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    else:
        p = to_device_batch(prev)
        w0, _, _, y0 = plan.solve(p["Ad"], p["Bd"], p["gd"], p["x0"], p["xref"], p["contact"], y_out=True)
        w, st, it, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                                  w_init=w0, y_init=y0, y_out=True)
    torch.cuda.synchronize()
    w = w.cpu().numpy()
    met = w[:, :3].copy()
    N = 16
    cs._B, cs._U = b, w[:, 12 * N:]
    t0 = time.time()
    with get_context("fork").Pool(16, initializer=cs._one_thread) as pool:
        res = list(pool.imap(cs._one, range(len(w)), chunksize=64))
    err = np.array([r[0] for r in res])
    kkt = np.array([r[1] for r in res])
    np.savez(out, err=err, kkt=kkt, gm=met[:, 0], cm=met[:, 1], us=met[:, 2],
             st=st.cpu().numpy(), it=it.cpu().numpy())
    print(f"{name}: certified in {time.time() - t0:.0f} s; status-1 max err {err[st.cpu().numpy() == 1].max():.3g}")


if __name__ == "__main__":
    main()
