"""Strong-scaling rehearsal on one GPU: time every rank's contiguous shard of the config-3
global batch (65,536) alone, for N = 1, 2, 4, 8 ranks (cmpc.dist.shard_bounds).  A multi-GPU
step takes as long as its slowest shard, so max over shards is the N-GPU step time."""
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
    from cmpc import _lib
    if len(sys.argv) > 1 and sys.argv[1]:
        _lib._lib = _lib.load(sys.argv[1])
    from cmpc import Plan, SolverParams, to_device_batch, synth
    from cmpc.dist import shard_bounds
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    # CMPC_PARAMS="name=value,...": other SolverParams overrides (A/B of runtime parameters)
    over = {k: type(getattr(SolverParams, k))(float(v)) for k, v in
            (a.split("=") for a in os.environ.get("CMPC_PARAMS", "").split(",") if a)}
    plan = Plan(SolverParams(**{"max_batch": 65536, **over}))
    if os.environ.get("CMPC_HEAVY_FIRST"):  # launch-order threshold (cmpc_plan_set_heavy_first)
        plan.set_heavy_first(int(os.environ["CMPC_HEAVY_FIRST"]))
    d = to_device_batch(synth.make_config(3))
    B = d["Ad"].shape[0]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for R in (1, 2, 4, 8):
        ms = []
        for r in range(R):
            lo, hi = shard_bounds(B, r, R)
            args = [d[k][lo:hi] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")]
            plan.solve(*args)
            torch.cuda.synchronize()
            t = []
            for _ in range(reps):
                ev0.record()
                plan.solve(*args)
                ev1.record()
                torch.cuda.synchronize()
                t.append(ev0.elapsed_time(ev1))
            ms.append(float(np.median(t)))
        print(f"N={R}: shard ms " + " ".join(f"{m:.2f}" for m in ms) +
              f" -> step {max(ms):.2f} ms, {B / max(ms) / 1e3:.2f} M solves/s")


if __name__ == "__main__":
    main()
