"""Diagnostic: when each instance of a batch starts and ends (libcmpc_times.so, built with
-DCMPC_DIAG_TIMES: status = start on the 100 MHz constant clock, iters = duration + 1e9 when the
instance finished in an elastic team).  Shows what sets the end of a batch: the slowest
instances, when they started, and whether the batch tail ran in team mode."""
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
    lib = sys.argv[1] if len(sys.argv) > 1 else str(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_times.so")
    _lib._lib = _lib.load(lib)
    from cmpc import Plan, SolverParams, to_device_batch, synth
    plan = Plan(SolverParams(max_batch=65536))
    cases = [(int(c), int(b)) for c, b in (a.split(":") for a in sys.argv[2:])] or \
        [(3, 8192), (2, 4096), (3, 16384), (3, 65536)]
    for cfg, B in cases:
        b = synth.make_config(cfg, B)
        d = to_device_batch(b)
        nc = 3 * (b["contact"].reshape(B, -1) != 0).sum(1)
        heavy = nc > 128
        # REPS back-to-back solves (as bench.py times them); the last one's timeline is shown
        w = torch.empty((B, 24 * 16), dtype=torch.float32, device="cuda")
        st = torch.empty((B,), dtype=torch.int32, device="cuda")
        it = torch.empty((B,), dtype=torch.int32, device="cuda")
        for rep in range(int(os.environ.get("REPS", "2"))):
            plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it),
                       stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        t0 = st.cpu().numpy().astype(np.int64)
        code = it.cpu().numpy().astype(np.int64)
        team = code >= 1000000000
        dur = code % 1000000000
        t0 = t0 - t0.min()
        t1 = t0 + dur
        end = t1.max()
        print(f"config {cfg} B {B}: batch {end / 100:.0f} us; teamed instances {team.sum()}")
        for name, m in (("light", ~heavy), ("heavy", heavy)):
            if m.any():
                print(f"  {name}: {m.sum()} inst, last end {t1[m].max() / 100:.0f} us, "
                      f"p50 end {np.percentile(t1[m], 50) / 100:.0f} us, mean dur {dur[m].mean() / 100:.1f} us, "
                      f"last start {t0[m].max() / 100:.0f} us")
        # concurrency: instances in flight of each class at 12 points of the batch (in group
        # mode the heavy count is the number of SIMDs the one-wave heavy class holds)
        pts = np.linspace(0, end, 14)[1:-1]
        for name, m in (("light", ~heavy), ("heavy", heavy)):
            if m.any():
                act = [int(np.sum(m & (t0 <= p) & (t1 > p))) for p in pts]
                print(f"  {name} in flight: " + " ".join(f"{a:5d}" for a in act))
        order = np.argsort(-t1)[:8]
        for i in order:
            print(f"    inst {i:6d} {'heavy' if heavy[i] else 'light'} nc {nc[i]:3d} start {t0[i] / 100:7.0f} us "
                  f"dur {dur[i] / 100:7.0f} us end {t1[i] / 100:7.0f} us team {int(team[i])}")


if __name__ == "__main__":
    main()
