"""Diagnostic: per-instance anatomy of every rank's shard of the config-3 global batch.
With libcmpc_times.so (-DCMPC_DIAG_TIMES) it records each instance's start and duration, with
libcmpc_diag.so (-DCMPC_DIAG_COUNTS) its ADMM iterations, polish sessions, factorizations and
wave cycles.  Saves <out>_<mode>.npz (one row per instance of the global batch, per N) and
prints what ends each shard: the last instances to finish, when they started, what they cost.
   usage: python tools/shard_anatomy.py times|counts OUT [N ...]"""
import functools
import sys
from pathlib import Path

import numpy as np

print = functools.partial(print, flush=True)
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    import torch
    from cmpc import _lib
    mode, out = sys.argv[1], sys.argv[2]
    Ns = [int(a) for a in sys.argv[3:]] or [1, 8]
    lib = {"times": "libcmpc_times.so", "counts": "libcmpc_diag.so"}[mode]
    _lib._lib = _lib.load(str(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib" / lib))
    from cmpc import Plan, SolverParams, to_device_batch, synth
    from cmpc.dist import shard_bounds
    plan = Plan(SolverParams(max_batch=65536))
    b = synth.make_config(3)
    d = to_device_batch(b)
    B = d["Ad"].shape[0]
    nc = 3 * (b["contact"].reshape(B, -1) != 0).sum(1)
    res = {"nc": nc}
    for R in Ns:
        a0 = np.zeros(B, np.int64)
        a1 = np.zeros(B, np.int64)
        for r in range(R):
            lo, hi = shard_bounds(B, r, R)
            args = [d[k][lo:hi] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")]
            for _ in range(2):  # the second (warm-cache) solve is the one kept
                w, st, it = plan.solve(*args)
            torch.cuda.synchronize()
            a0[lo:hi] = st.cpu().numpy()
            a1[lo:hi] = it.cpu().numpy()
            if mode == "times":
                t0 = a0[lo:hi] - a0[lo:hi].min()
                t1 = t0 + a1[lo:hi] % 1000000000
                last = np.argsort(-t1)[:4]
                print(f"N={R} shard {r}: end {t1.max() / 100:.0f} us; last: " + "; ".join(
                    f"{lo + i} nc {nc[lo + i]} start {t0[i] / 100:.0f} dur {(t1[i] - t0[i]) / 100:.0f}"
                    for i in last))
            else:
                cyc = a0[lo:hi] * 16
                top = np.argsort(-cyc)[:4]
                code = a1[lo:hi]
                print(f"N={R} shard {r}: mean {cyc.mean():.0f} cyc; top: " + "; ".join(
                    f"{lo + i} cyc {cyc[i]} it {code[i] % 1000} pol {(code[i] // 1000) % 1000} "
                    f"fact {code[i] // 1000000}" for i in top))
        res[f"a0_{R}"] = a0
        res[f"a1_{R}"] = a1
    np.savez_compressed(f"{out}_{mode}.npz", **res)


if __name__ == "__main__":
    main()
