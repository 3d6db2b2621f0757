"""A/B of two library builds for bit-identical results: solve the headline batch (config 3,
65,536) cold and its next tick warm, config 2 at 4,096 cold, with the library given, and write a
digest of (w, status, iterations); run once per library in separate processes, then compare.
    python tools/bitwise_ab.py LIB OUT.npz            (GPU)
    python tools/bitwise_ab.py --compare A.npz B.npz   (CPU)"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def run(lib, out):
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(lib)
    from cmpc import Plan, SolverParams, to_device_batch, synth
    plan = Plan(SolverParams(max_batch=65536))
    res = {}
    for tag, b, prev in (("cfg3", synth.make_config(3), None),
                         ("cfg2", synth.make_config(2, B=4096), None),
                         ("cfg3_next_warm", synth.next_tick(synth.make_config(3)), synth.make_config(3))):
        kw = {}
        if prev is not None:
            dp = to_device_batch(prev)
            y = torch.empty((dp["Ad"].shape[0], 12 * 16), dtype=torch.float32, device=dp["Ad"].device)
            w0, _, _ = plan.solve(*(dp[k] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")), y_out=y)
            kw = dict(w_init=w0, y_init=y)
        d = to_device_batch(b)
        w, st, it = plan.solve(*(d[k] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")), **kw)
        torch.cuda.synchronize()
        res[tag + "_w"] = w.cpu().numpy()
        res[tag + "_st"] = st.cpu().numpy()
        res[tag + "_it"] = it.cpu().numpy()
    np.savez_compressed(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32) if A[k].dtype == np.float32 else A[k],
                              B[k].view(np.uint32) if B[k].dtype == np.float32 else B[k])
        nd = int(np.sum(np.any((A[k] != B[k]).reshape(A[k].shape[0], -1), axis=1)))
        print(f"{k}: {'bit-identical' if same else f'{nd} instances differ'}")
        ok = ok and same
    print("ALL BIT-IDENTICAL" if ok else "DIFFERENT")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], sys.argv[2])
