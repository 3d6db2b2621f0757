"""Parity evidence beyond the committed fixtures (test infrastructure, not collected by pytest):
a random sample of the headline batch (config 3, 65,536) solved by the HIP path on the GPU box,
then every sampled instance certified on the CPU against its KKT-certified optimum
(oracle/tight_solver.py) and the distribution of max|dU|/max|U| reported.

    python tests/certify_sample.py gpu [--n 4096]   # on the GPU box: gpurun_out/w_sample.npz
    python tests/certify_sample.py cpu [--limit 512] # here: the report (profiles/r04f_parity_sample.txt;
                                                      # ~3 s of CPU per instance)
"""
import argparse
import sys
from multiprocessing import Pool
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tests"), str(REPO), str(REPO / "convex-mpc-unitree-go2_amd")]
OUT = REPO / "gpurun_out" / "w_sample.npz"
_B = None


def gpu(n):
    import torch
    from cmpc import Plan, SolverParams, synth, to_device_batch
    b = synth.make_config(3, B=65536)
    plan = Plan(SolverParams(max_batch=65536))
    d = to_device_batch(b)
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()
    idx = np.sort(np.random.default_rng(2026).choice(65536, n, replace=False))
    OUT.parent.mkdir(exist_ok=True)
    np.savez_compressed(OUT, idx=idx, w=w.cpu().numpy()[idx], st=st.cpu().numpy()[idx],
                        it=it.cpu().numpy()[idx])
    print("saved", OUT, len(idx))


def _one(i):
    from oracle import mpc_qp, tight_solver
    qp = mpc_qp.build_qp(_B["Ad"][i], _B["Bd"][i], _B["gd"][i], _B["x0"][i], _B["xref"][i].T,
                         _B["contact"][i])
    r = tight_solver.solve(qp)
    return r["w"], max(r["kkt"].values())


def cpu(limit):
    global _B
    from cmpc import synth
    from parity_util import rel_err_U
    _B = synth.make_config(3, B=65536)
    z = dict(np.load(OUT))
    if limit and limit < len(z["idx"]):  # every k-th of the saved random sample
        k = len(z["idx"]) // limit
        z = {key: v[::k][:limit] for key, v in z.items()}
    idx = z["idx"]
    with Pool(8) as pool:
        res = pool.map(_one, idx.tolist(), chunksize=16)
    wopt = np.stack([r[0] for r in res])
    kkt = np.array([r[1] for r in res])
    err = rel_err_U(z["w"], wopt)
    nf = 3 * (_B["contact"][idx] != 0).reshape(len(idx), -1).sum(1)
    bins = np.searchsorted(np.array([96, 128, 144, 160, 192]), nf)
    print(f"config 3 (65,536, one solve): {len(idx)} random instances (seed 2026) against their "
          f"KKT-certified optimum (max KKT residual {kkt.max():.1e}); status 1: {np.mean(z['st'] == 1):.4f}")
    print(f"max|dU| / max|U|: median {np.median(err):.2e}  p90 {np.quantile(err, .9):.2e}  "
          f"p99 {np.quantile(err, .99):.2e}  p99.9 {np.quantile(err, .999):.2e}  max {err.max():.2e}")
    print(f"above the 1e-4 bar: {int((err > 1e-4).sum())} of {len(idx)}; above 5e-5: {int((err > 5e-5).sum())}")
    for q in range(5):
        m = bins == q
        if m.any():
            print(f"  bin NC {[96, 128, 144, 160, 192][q]:3d}: {int(m.sum()):5d} instances, max {err[m].max():.2e}")
    worst = np.argsort(-err)[:5]
    print("worst:", ", ".join(f"{int(idx[k])} ({err[k]:.2e}, {int(z['it'][k])} it)" for k in worst))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("gpu", "cpu"))
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--limit", type=int, default=0, help="cpu: certify this many of the saved sample")
    a = ap.parse_args()
    gpu(a.n) if a.mode == "gpu" else cpu(a.limit)
