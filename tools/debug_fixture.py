"""Diagnostic: per-instance status / iterations / error of the GPU solver on a golden fixture,
next to the NumPy model of the algorithm (tests/algo_spec.py)."""
import argparse
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))
sys.path.insert(0, str(REPO / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="qp_cfg1.npz")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--spec", action="store_true")
    a = ap.parse_args()
    from cmpc import _lib
    if a.lib:
        _lib._lib = _lib.load(Path(a.lib))
    from cmpc import solve_batch, Plan, SolverParams
    from parity_util import load_fixture, fixture_batch, rel_err_U
    fx = load_fixture(a.fixture)
    batch = fixture_batch(fx)
    plan = Plan(SolverParams(max_batch=4096))
    w, st, it = solve_batch(batch, plan=plan)
    err = rel_err_U(w, fx["w"])
    for i in range(len(st)):
        line = f"{i:3d} status {st[i]:4d} iters {it[i]:5d} relerr {err[i]:.2e}"
        if a.spec:
            import algo_spec
            out = algo_spec.solve({k: v[i] for k, v in batch.items()}, algo_spec.Params())
            line += f"   spec: status {out['status']} iters {out['iters']}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
