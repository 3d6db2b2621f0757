"""Diagnostic: cfg2 throughput / iteration tail as a function of polish repairs."""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import Plan, SolverParams, to_device_batch, synth
    b = synth.make_batch(65536, seed=2, mixed=True)
    d = to_device_batch(b)
    for rep in (3, 6, 10, 16):
        for stable in (3, 2):
            plan = Plan(SolverParams(max_batch=65536, polish_repairs=rep, polish_stable=stable))
            w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            itn = it.cpu().numpy()
            stn = st.cpu().numpy()
            print(f"repairs {rep:2d} stable {stable}: {65536 / dt / 1e6:6.3f} M/s  iters mean {itn.mean():.2f} "
                  f"p99 {np.percentile(itn, 99):.0f} max {itn.max()}  >50: {(itn > 50).sum()}  "
                  f"solved {(stn == 1).mean():.5f}", flush=True)


if __name__ == "__main__":
    main()
