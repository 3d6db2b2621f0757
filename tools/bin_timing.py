"""Diagnostic: throughput of the product solver on single-bin subsets of the synthetic configs."""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import Plan, SolverParams, to_device_batch, synth
    caps = np.array([96, 128, 160, 192])
    plan = Plan(SolverParams(max_batch=65536))
    for cfg, mixed in ((1, False), (2, True)):
        # a large draw so that every bin holds up to 65,536 instances of its own (per-instance
        # cost at full load, not a tail of a few instances per wave)
        Bd = 65536 if cfg == 1 else 262144
        b = synth.make_batch(Bd, seed=cfg, mixed=mixed)
        nf = 3 * (b["contact"] != 0).reshape(Bd, -1).sum(1)
        binq = np.searchsorted(caps, nf)
        for q in range(4):
            keep = binq == q
            keep &= np.cumsum(keep) <= 65536
            cnt = int(keep.sum())
            if cnt < 512:
                continue
            sub = {k: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == keep.shape else v)
                   for k, v in b.items()}
            d = to_device_batch(sub)
            for _ in range(2):
                w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 5
            itn = it.cpu().numpy()
            print(f"cfg{cfg} bin{caps[q]} n={cnt:6d}  {cnt / dt / 1e6:6.3f} M solves/s  iters mean "
                  f"{itn.mean():.2f} max {itn.max()}  solved {(st.cpu().numpy() == 1).mean():.4f}  "
                  f"nf mean {nf[keep].mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
