"""Diagnostic: the worst primal-feasibility instances of a batch (reference bounds / friction
rows, tests/parity_util.feasibility) for a library build.
   python tools/feas_check.py lib.so [config] [B]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))
sys.path.insert(0, str(REPO / "tests"))


def main():
    from cmpc import _lib
    _lib._lib = _lib.load(sys.argv[1])
    from cmpc import Plan, SolverParams, solve_batch, synth
    from parity_util import split_w, feasibility
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    b = synth.make_config(cfg, B=B)
    w, st, it = solve_batch(b, plan=Plan(SolverParams(max_batch=B)))
    _, U = split_w(w.astype(np.float64))
    f = feasibility(b, U)
    nf = 3 * (b["contact"] != 0).reshape(B, -1).sum(1)
    order = np.argsort(-f)[:6]
    print(Path(sys.argv[1]).name, "max violation", f.max(), "status", np.unique(st, return_counts=True))
    for i in order:
        F = U[i].reshape(16, 4, 3)
        ct = b["contact"][i].T.astype(bool)
        v = np.maximum.reduce([10.0 - F[..., 2], np.abs(F[..., 0]) - 0.8 * F[..., 2],
                               np.abs(F[..., 1]) - 0.8 * F[..., 2]]) * ct
        k, l = np.unravel_index(np.argmax(v), v.shape)
        print(f"  inst {i} n {nf[i]} iters {it[i]} viol {f[i]:.4g} at step {k} leg {l} force {F[k, l]}")


if __name__ == "__main__":
    main()
