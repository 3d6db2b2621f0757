"""Lagrange multipliers of the reference QP recovered from the primal solution.

The single-robot ``CentroidalMPC.solve_QP`` API returns ``sol["lam_x"]`` / ``sol["lam_a"]``
(centroidal_mpc.py:108-110) in CasADi's convention  H w + g + A' lam_a + lam_x = 0  with
lam > 0 on active upper bounds, lam < 0 on active lower bounds.  Given the GPU's primal w they
follow in closed form (host-side post-processing of one instance, not part of the batched
hot path):

* dynamics rows (centroidal_mpc.py:287-303): stationarity in x_j gives the backward
  recursion lam_a[j-1] = Ad' lam_a[j] - 2Q (x_j - xref_{j-1}), lam_a[N] = 0;
* per stance (step, leg): s = 2R u_k - Bd_k' lam_a[k] restricted to the leg must equal
  -(F' lam_fric + lam_x); the active friction faces / fz bound are read off u and their
  multipliers solved from the 3 components (the same relations the kernel's KKT check uses);
* swing legs: lam_x = -s (equality bounds), friction multipliers 0 (rows are free).
"""
from __future__ import annotations

import numpy as np


def recover(Ad, Bd, gd, x0, xref, contact, w, Q, R, mu, fz_min, tol=1e-6):
    """Ad (12,12), Bd (N,12,12), xref (N,12) rows = targets of x_{k+1}, contact (4,N),
    w (24N,) reference layout -> lam_x (24N,), lam_a (28N,)."""
    N = Bd.shape[0]
    Qd = np.diag(Q) if np.ndim(Q) == 2 else np.asarray(Q)
    Rd = np.diag(R) if np.ndim(R) == 2 else np.asarray(R)
    X = w[:12 * N].reshape(N, 12)
    U = w[12 * N:].reshape(N, 12)
    nu = np.zeros((N + 1, 12))
    for j in range(N, 0, -1):
        nu[j - 1] = Ad.T @ nu[j] - 2.0 * Qd * (X[j - 1] - xref[j - 1])
    lam_eq = nu[:N]
    lam_fric = np.zeros((N, 4, 4))
    lam_x = np.zeros(24 * N)
    for k in range(N):
        s = 2.0 * Rd * U[k] - Bd[k].T @ lam_eq[k]
        for leg in range(4):
            sl = s[3 * leg:3 * leg + 3]
            base = 12 * N + 12 * k + 3 * leg
            if not contact[leg, k]:
                lam_x[base:base + 3] = -sl
                continue
            fx, fy, fz = U[k, 3 * leg:3 * leg + 3]
            scale = tol * max(1.0, abs(fz))
            lf = np.zeros(4)
            # face rows: [fx - mu fz, -fx - mu fz, fy - mu fz, -fy - mu fz] <= 0
            if abs(fx - mu * fz) <= scale:
                lf[0] = max(-sl[0], 0.0)
            elif abs(fx + mu * fz) <= scale:
                lf[1] = max(sl[0], 0.0)
            if abs(fy - mu * fz) <= scale:
                lf[2] = max(-sl[1], 0.0)
            elif abs(fy + mu * fz) <= scale:
                lf[3] = max(sl[1], 0.0)
            lam_fric[k, leg] = lf
            rz = sl[2] - mu * lf.sum()          # = -lam_x[fz]
            if abs(fz - fz_min) <= scale:
                lam_x[base + 2] = min(-rz, 0.0)  # active lower bound -> negative multiplier
    lam_a = np.concatenate([lam_eq.reshape(-1), lam_fric.reshape(-1)])
    return lam_x, lam_a


def cost(w, xref, Q, R):
    """½ w'Hw + g'w of the reference (H = diag(2Q, 2R), g = [-2Q xref; 0])."""
    N = xref.shape[0]
    Qd = np.diag(Q) if np.ndim(Q) == 2 else np.asarray(Q)
    Rd = np.diag(R) if np.ndim(R) == 2 else np.asarray(R)
    X = w[:12 * N].reshape(N, 12)
    U = w[12 * N:].reshape(N, 12)
    return float(np.sum(Qd * X * X) + np.sum(Rd * U * U) - 2.0 * np.sum(Qd * xref * X))
