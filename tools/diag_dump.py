"""Diagnostic: per-instance cycles / iterations / factorizations of the cfg2 batch (diag build),
saved with the batch's contact tables for offline analysis (gpurun_out/diag_cfg2.npz)."""
import sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_diag.so")
    from cmpc import Plan, SolverParams, to_device_batch, synth
    plan = Plan(SolverParams(max_batch=65536))
    b = synth.make_batch(65536, seed=2, mixed=True)
    d = to_device_batch(b)
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()
    cyc = st.cpu().numpy().astype(np.int64) * 16
    code = it.cpu().numpy().astype(np.int64)
    np.savez_compressed(REPO / "gpurun_out/diag_cfg2.npz", cycles=cyc, iters=code % 1000,
                        polish=(code // 1000) % 1000, fact=code // 1000000)
    print("saved", cyc.mean())


if __name__ == "__main__":
    main()
