"""Debug: compare cmpc_solve_warm's y_out with -grad f(U) of the reference QP (numeric, float64)
for one instance of a synthetic batch.  usage: python tools/dual_debug.py [cfg] [B] [index]"""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "convex-mpc-unitree-go2_amd")]
from cmpc import Plan, SolverParams, synth  # noqa: E402
from cmpc.solver import to_device_batch  # noqa: E402
from oracle import mpc_qp  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
i = int(sys.argv[3]) if len(sys.argv) > 3 else 442
b = synth.make_config(cfg, B=B)
plan = Plan(SolverParams(max_batch=B))
d = to_device_batch(b, plan.device)
w, st, it, y = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], y_out=True)
torch.cuda.synchronize()
w, y = w.cpu().numpy().astype(np.float64), y.cpu().numpy().astype(np.float64)
if i < 0:
    i = int(np.abs(y).max(1).argmax())
print("instance", i, "status", int(st[i]), "iters", int(it[i]), "batch max|y| %.4g" % np.abs(y).max(),
      "instance max|y| %.4g" % np.abs(y[i]).max())
qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                     b["contact"][i])
N = 16
U = w[i, 12 * N:].reshape(N, 12)


def f(U):
    X = mpc_qp.rollout(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], U)
    ww = mpc_qp.pack_w(X, U)
    return 0.5 * ww @ (qp["h"] @ ww) + qp["g"] @ ww


ct = b["contact"][i].T.astype(bool)  # (N, 4)
grad = np.zeros((N, 12))
h = 1e-2
for k in range(N):
    for l in range(4):
        if not ct[k, l]:
            continue
        for a in range(3):
            e = np.zeros((N, 12)); e[k, 3 * l + a] = h
            grad[k, 3 * l + a] = (f(U + e) - f(U - e)) / (2 * h)
Y = y[i].reshape(N, 12)
mask = np.repeat(ct, 3, axis=1)
r = (-grad[mask]) / np.where(np.abs(Y[mask]) > 0, Y[mask], np.nan)
print("ratio -grad/y: median %.4g  min %.4g  max %.4g" % (np.nanmedian(r), np.nanmin(r),
                                                          np.nanmax(r)))
np.set_printoptions(precision=4, suppress=False, linewidth=160)
for k in range(N):
    for l in range(4):
        if ct[k, l]:
            print(k, l, "u", U[k, 3 * l:3 * l + 3], "y", Y[k, 3 * l:3 * l + 3],
                  "-g", -grad[k, 3 * l:3 * l + 3])
