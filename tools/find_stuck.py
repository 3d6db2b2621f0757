"""Diagnostic: instances of a cfg batch (seed offset argv[1], lib argv[2], config argv[3],
default 2) that do not reach status 1, with their
iteration / polish-session / factorization counts (product and diag builds)."""
import sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    if len(sys.argv) > 2:  # alternative build
        _lib._lib = _lib.load(sys.argv[2])
    from cmpc import Plan, SolverParams, to_device_batch, synth
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    seed = synth.CONFIGS[cfg]["seed"] + int(sys.argv[1])
    b = synth.make_batch(65536, seed=seed, mixed=synth.CONFIGS[cfg]["mixed"])
    d = to_device_batch(b)
    plan = Plan(SolverParams(max_batch=65536))
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()
    st, it = st.cpu().numpy(), it.cpu().numpy()
    bad = np.nonzero(st != 1)[0]
    print("seed", seed, "not status 1:", bad.tolist(), st[bad].tolist(), it[bad].tolist())
    print("iterations: mean %.3f sum %d" % (it.mean(), it.sum()))
    top = np.argsort(-it)[:6]
    print("most iterations:", top.tolist(), it[top].tolist())
    np.save(REPO / "gpurun_out/stuck_idx.npy", np.concatenate([bad, top]))


if __name__ == "__main__":
    main()
