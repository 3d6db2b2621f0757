"""Diagnostic: run a cfg2 batch (seed offset argv[1]) through libcmpc_trace.so (-DCMPC_TRACE=<b>),
which printf-traces instance b's ADMM iterations and polish sessions."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_trace.so")
    from cmpc import Plan, SolverParams, to_device_batch, synth
    b = synth.make_batch(65536, seed=2 + int(sys.argv[1]), mixed=True)
    d = to_device_batch(b)
    plan = Plan(SolverParams(max_batch=65536))
    plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
