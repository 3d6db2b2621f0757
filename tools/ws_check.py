"""Diagnostic: status / iteration statistics of the large-batch solve kernels on the benchmark
batches, wrench-space (default) vs n-space (CMPC_SOLVE_KERNEL=group) plans, and the instances
that end with a status other than 1."""
import functools
import os
import sys
from pathlib import Path

import numpy as np

print = functools.partial(print, flush=True)
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import Plan, SolverParams, solve_batch, synth
    over = dict(a.split("=") for a in sys.argv[1:] if "=" in a)
    over = {k: type(getattr(SolverParams, k))(float(v) if "." in v else int(v)) for k, v in over.items()}
    plans = {}
    for mode in ("ws", "group"):
        if mode == "group":
            os.environ["CMPC_SOLVE_KERNEL"] = "group"
        plans[mode] = Plan(SolverParams(max_batch=65536, **over))
        os.environ.pop("CMPC_SOLVE_KERNEL", None)
    for cfg, B in ((3, 65536), (2, 65536), (1, 65536), (2, 4096), (3, 8192)):
        b = synth.make_config(cfg, B=B) if cfg == 3 else synth.make_batch(B, seed=cfg, mixed=cfg == 2)
        nf = 3 * (b["contact"].reshape(B, -1) != 0).sum(1)
        res = {}
        for mode, plan in plans.items():
            w, st, it = solve_batch(b, plan=plan)
            res[mode] = (w, st, it)
            u, c = np.unique(st, return_counts=True)
            print(f"cfg {cfg} B {B} {mode:5s} {plan.solve_kernels(B)[0]}: status {dict(zip(u.tolist(), c.tolist()))} "
                  f"iters mean {it.mean():.2f} p99 {np.percentile(it, 99):.0f} max {it.max()}")
        w, st, it = res["ws"]
        w0, st0, it0 = res["group"]
        U, U0 = w[:, 192:].astype(np.float64), w0[:, 192:].astype(np.float64)
        d = np.abs(U - U0).max(1) / np.maximum(np.abs(U0).max(1), 1e-12)
        print(f"   ws vs group: max rel dU {d.max():.2e} (p99.9 {np.percentile(d, 99.9):.2e}); "
              f"iters ws-group mean {np.mean(it.astype(float) - it0):+.2f}")
        bins = np.searchsorted(np.array([96, 128, 160, 192]), nf)
        for q, cap in enumerate((96, 128, 160, 192)):
            m = bins == q
            if m.any():
                print(f"   bin {cap}: {m.sum()} inst, ws not-1 {int(np.sum(st[m] != 1))}, ws iters mean "
                      f"{it[m].mean():.2f} vs group {it0[m].mean():.2f}")
        bad = np.flatnonzero(st != 1)[:12]
        for i in bad:
            print(f"   inst {i}: ws status {st[i]} iters {it[i]} | group status {st0[i]} iters {it0[i]} | nf {nf[i]} "
                  f"dU {d[i]:.2e}")


if __name__ == "__main__":
    main()
