"""Why the wrench-space (Woodbury) factorization was not adopted: quality of the
fp32 preconditioner M ~ (H + shift)^-1 as the spectral radius of I - M H, on the committed
fixtures, for
  * the n-space inverse the kernels use (fp32 condensation + fp32 inverse), and
  * Woodbury in the wrench space: H + shift = D + V' Pw V (Bd_k = Mb E_k, Mb = [1/2 Ad[0:6, 6:12]; I6]),
    M = D^-1 - D^-1 V' W V D^-1, W = (Pw^-1 + V D^-1 V')^-1, with the pieces rounded to fp32 one at
    a time ('W32': only W rounded -- already enough to lose the preconditioner).
   usage: python tools/wrench_precond.py [qp_cfg2.npz qp_hard.npz ...]"""
import sys
from pathlib import Path

import numpy as np
import scipy.linalg as sl

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tests"), str(REPO)]
from parity_util import load_fixture, fixture_batch  # noqa: E402

F = np.float32
Q = np.array([1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1], np.float64)
R = np.full(12, 1e-5)
MU, FZ = 0.8, 10.0


def inv32(H):
    c, low = sl.cho_factor(H.astype(F), lower=True)
    return sl.cho_solve((c, low), np.eye(H.shape[0], dtype=F)).astype(F)


def condense(A, Bt, Q2, dtype):
    N = len(Bt)
    off = np.concatenate([[0], np.cumsum([b.shape[1] for b in Bt])]).astype(int)
    n = off[-1]
    H = np.zeros((n, n), dtype)
    Gt = np.zeros((12, n), dtype)
    for t in range(N):
        Gt = A @ Gt
        Gt[:, off[t]:off[t + 1]] = Bt[t]
        H += Gt.T @ (Q2[:, None].astype(dtype) * Gt)
    return H


def face_basis(inst, w):
    """per-step reduced columns T_k and weights of the certified optimum's face set"""
    ct = inst["contact"]
    N = ct.shape[1]
    U = w[192:].reshape(N, 12)
    Ts, Rs = [], []
    for k in range(N):
        cols, rr = [], []
        for leg in range(4):
            if not ct[leg, k]:
                continue
            fx, fy, fz = U[k, 3 * leg:3 * leg + 3]
            tol = 1e-6 * max(1, abs(fz))
            sx = 1 if fx >= MU * fz - tol else (-1 if fx <= -MU * fz + tol else 0)
            sy = 1 if fy >= MU * fz - tol else (-1 if fy <= -MU * fz + tol else 0)
            b = 3 * leg
            if sx == 0:
                e = np.zeros(12); e[b] = 1; cols.append(e); rr.append(R[b])
            if sy == 0:
                e = np.zeros(12); e[b + 1] = 1; cols.append(e); rr.append(R[b + 1])
            if fz > FZ + tol:
                e = np.zeros(12); e[b + 2] = 1; e[b] = sx * MU; e[b + 1] = sy * MU; cols.append(e)
                rr.append(R[b + 2] + MU * MU * ((sx != 0) * R[b] + (sy != 0) * R[b + 1]))
        Ts.append(np.array(cols).T if cols else np.zeros((12, 0)))
        Rs.append(np.array(rr))
    return Ts, np.concatenate(Rs)


def radii(inst, w, shift=1e-6):
    A = inst["Ad"].astype(np.float64)
    B = inst["Bd"].astype(np.float64)
    N = B.shape[0]
    Ts, Rt = face_basis(inst, w)
    Bt = [B[k] @ Ts[k] for k in range(N)]
    n = sum(t.shape[1] for t in Ts)
    H = condense(A, Bt, 2 * Q, np.float64) + np.diag(2 * Rt + shift)
    rho = lambda M: float(np.max(np.abs(np.linalg.eigvals(np.eye(n) - M @ H))))  # noqa: E731
    out = {}
    H32 = condense(A.astype(F), [b.astype(F) for b in Bt], (2 * Q).astype(F), F) + np.diag((2 * Rt + shift).astype(F))
    out["n-space fp32"] = rho(inv32(H32).astype(np.float64))
    Mb = np.vstack([0.5 * A[0:6, 6:12], np.eye(6)])
    E = [b[6:12] for b in Bt]
    Pti = np.linalg.inv(condense(A, [Mb] * N, 2 * Q, np.float64))
    Dinv = 1 / (2 * Rt + shift)
    off = np.concatenate([[0], np.cumsum([e.shape[1] for e in E])]).astype(int)
    S = np.zeros((6 * N, 6 * N))
    V = np.zeros((6 * N, n))
    for k in range(N):
        V[6 * k:6 * k + 6, off[k]:off[k + 1]] = E[k]
        S[6 * k:6 * k + 6, 6 * k:6 * k + 6] = (E[k] * Dinv[off[k]:off[k + 1]][None, :]) @ E[k].T
    W = np.linalg.inv(Pti + S)
    wood = lambda W_: np.diag(Dinv) - (Dinv[:, None] * V.T) @ W_ @ (V * Dinv[None, :])  # noqa: E731
    out["Woodbury fp64"] = rho(wood(W))
    out["Woodbury W32"] = rho(wood(W.astype(F).astype(np.float64)))
    out["Woodbury Pw^-1 fp32"] = rho(wood(np.linalg.inv(Pti.astype(F).astype(np.float64) + S)))
    return out


def main():
    res = {}
    for name in (sys.argv[1:] or ["qp_cfg2.npz", "qp_hard.npz"]):
        fx = load_fixture(name)
        b = fixture_batch(fx)
        for i in range(min(len(fx["w"]), 24)):
            for k, v in radii({k: v[i] for k, v in b.items()}, fx["w"][i]).items():
                res.setdefault(k, []).append(v)
    for k, v in res.items():
        v = np.array(v)
        print(f"{k:22s} rho(I - M H): median {np.median(v):.1e}  p90 {np.percentile(v, 90):.1e}  max {v.max():.1e}")


if __name__ == "__main__":
    main()
