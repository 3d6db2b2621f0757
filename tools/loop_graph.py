"""Diagnostic: the closed-loop tick (cmpc/closed_loop.py) eager vs HIP-graph replay on the same
tick sequence -- per-tick wall time of each mode, for rocprofv3 kernel traces of both.
   usage: python tools/loop_graph.py [B] [ticks] [lib] [modes: eager,graph,eager2,graph2,graphsync]"""
import functools
import sys
import time
from pathlib import Path

import numpy as np

print = functools.partial(print, flush=True)
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    if len(sys.argv) > 3 and sys.argv[3]:
        _lib._lib = _lib.load(sys.argv[3])
    from cmpc import Plan, SolverParams
    from cmpc.closed_loop import ClosedLoop
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    plan = Plan(SolverParams(max_batch=max(B, 1024)))
    rg = np.random.default_rng(100)
    cmd = np.stack([rg.uniform(-0.5, 0.5, B), rg.uniform(-0.2, 0.2, B), np.full(B, 0.27),
                    rg.uniform(-1, 1, B)], 1)
    res = {}
    modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["eager", "graph", "eager2", "graph2"]
    for mode in modes:
        cl = ClosedLoop(B, plan=plan, seed=0)
        cl.set_command(cmd)
        for _ in range(4):
            cl.tick()
        if mode.startswith("graph"):
            cl.capture()  # records tick 5 without running it
        cl.tick()  # tick 5 (the graph's first replay): both modes then time ticks 6 .. 5 + T
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(T):
            cl.tick()
            if mode.endswith("sync"):  # no replay queued behind the running one
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res[mode] = el / T * 1e3
        print(f"B {B} {mode}: {el / T * 1e3:.3f} ms per tick, {B * T / el / 1e6:.2f} M robot-ticks/s, "
              f"iters mean {cl.iters.float().mean().item():.3f}")
        del cl


if __name__ == "__main__":
    main()
