"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- KKT-certified float64 solve of the reference QP.

The reference solves its QP with CasADi 3.6.7's OSQP plugin (``centroidal_mpc.py:213``,
called at ``:98``).  Neither CasADi nor OSQP exists in this image, so the QP *solution* cannot
be compared with the reference's own output.  The QP is strictly convex (H is diagonal
positive, ``centroidal_mpc.py:178-201``) and always feasible, so its optimum is unique; this
module computes that optimum in the reference's own variable/constraint layout with a dense
primal-dual interior-point method (Mehrotra predictor-corrector) followed by an exact
active-set polish, and returns the KKT residuals that certify it.  That certified optimum is
the parity target for the HIP solver.

Multipliers follow the CasADi conic convention: H w + g + A^T lam_a + lam_x = 0 with
lam > 0 on active upper bounds and lam < 0 on active lower bounds.
"""
from __future__ import annotations

import numpy as np

from . import mpc_qp


def _split_constraints(qp):
    A = qp['a'].toarray()
    n = A.shape[1]
    lba, uba, lbx, ubx = qp['lba'], qp['uba'], qp['lbx'], qp['ubx']
    E_rows, b, eq_map = [], [], []     # eq_map: ('a'|'x', index, sign)
    G_rows, h, in_map = [], [], []
    I = np.eye(n)
    for r in range(A.shape[0]):
        lo, hi = lba[r], uba[r]
        if np.isfinite(lo) and np.isfinite(hi) and lo == hi:
            E_rows.append(A[r]); b.append(hi); eq_map.append(('a', r, 1.0))
            continue
        if np.isfinite(hi):
            G_rows.append(A[r]); h.append(hi); in_map.append(('a', r, 1.0))
        if np.isfinite(lo):
            G_rows.append(-A[r]); h.append(-lo); in_map.append(('a', r, -1.0))
    for i in range(n):
        lo, hi = lbx[i], ubx[i]
        if np.isfinite(lo) and np.isfinite(hi) and lo == hi:
            E_rows.append(I[i]); b.append(hi); eq_map.append(('x', i, 1.0))
            continue
        if np.isfinite(hi):
            G_rows.append(I[i]); h.append(hi); in_map.append(('x', i, 1.0))
        if np.isfinite(lo):
            G_rows.append(-I[i]); h.append(-lo); in_map.append(('x', i, -1.0))
    return (np.array(E_rows).reshape(-1, n), np.array(b, dtype=float), eq_map,
            np.array(G_rows).reshape(-1, n), np.array(h, dtype=float), in_map)


def _to_casadi_duals(n, m, nu, lam, eq_map, in_map):
    lam_x = np.zeros(n)
    lam_a = np.zeros(m)
    for v, (kind, idx, sgn) in zip(nu, eq_map):
        (lam_a if kind == 'a' else lam_x)[idx] += sgn * v
    for v, (kind, idx, sgn) in zip(lam, in_map):
        (lam_a if kind == 'a' else lam_x)[idx] += sgn * v
    return lam_x, lam_a


def solve(qp, tol: float = 1e-13, max_iter: int = 80, polish: bool = True):
    """Solve the reference QP to a certified optimum.

    Returns dict(w, lam_x, lam_a, iters, kkt) where kkt = mpc_qp.kkt_residuals(...).
    """
    H = qp['h'].toarray()
    g = qp['g']
    n = H.shape[0]
    m = qp['a'].shape[0]
    E, b, eq_map, G, h, in_map = _split_constraints(qp)
    me, mi = E.shape[0], G.shape[0]
    if mi == 0:  # equality-constrained only (e.g. every leg in swing): one KKT solve
        K = np.zeros((n + me, n + me))
        K[:n, :n] = H
        K[:n, n:] = E.T
        K[n:, :n] = E
        sol = np.linalg.solve(K, np.concatenate([-g, b]))
        lam_x, lam_a = _to_casadi_duals(n, m, sol[n:], np.zeros(0), eq_map, in_map)
        return dict(w=sol[:n], lam_x=lam_x, lam_a=lam_a, iters=0,
                    kkt=mpc_qp.kkt_residuals(qp, sol[:n], lam_x, lam_a), polished=True)

    w = np.zeros(n)
    nu = np.zeros(me)
    s = np.ones(mi)
    lam = np.ones(mi)
    # start: satisfy equalities via least-norm, slacks positive
    w = np.linalg.lstsq(E, b, rcond=None)[0] if me else w
    r0 = h - G @ w
    s = np.maximum(r0, 1.0)
    lam = np.ones(mi)

    it = 0
    for it in range(1, max_iter + 1):
        rd = H @ w + g + E.T @ nu + G.T @ lam
        re = E @ w - b
        ri = G @ w + s - h
        mu = s @ lam / mi
        if (np.max(np.abs(rd)) < tol * (1 + np.max(np.abs(g))) and
                np.max(np.abs(re), initial=0) < tol * (1 + np.max(np.abs(b))) and
                np.max(np.abs(ri)) < tol * (1 + np.max(np.abs(h))) and mu < tol):
            break
        Wd = lam / s
        K = np.zeros((n + me, n + me))
        K[:n, :n] = H + G.T @ (Wd[:, None] * G)
        K[:n, n:] = E.T
        K[n:, :n] = E
        # tiny regularisation on the equality block keeps K non-singular when the
        # swing-fix rows and dynamics rows are dependent (they are not, but be safe)
        K[n:, n:] = -1e-14 * np.eye(me)

        def step(rc):
            rhs = np.concatenate([-rd + G.T @ ((rc - lam * ri) / s), -re])
            sol = np.linalg.solve(K, rhs)
            dw = sol[:n]
            dnu = sol[n:]
            ds = -ri - G @ dw
            dlam = (-rc - lam * ds) / s
            return dw, dnu, ds, dlam

        def max_step(v, dv):
            neg = dv < 0
            if not np.any(neg):
                return 1.0
            return min(1.0, float(np.min(-v[neg] / dv[neg])))

        # predictor (affine)
        dw, dnu, ds, dlam = step(s * lam)
        a_aff = min(max_step(s, ds), max_step(lam, dlam))
        mu_aff = (s + a_aff * ds) @ (lam + a_aff * dlam) / mi
        sigma = (mu_aff / mu) ** 3
        # corrector
        rc = s * lam + ds * dlam - sigma * mu
        dw, dnu, ds, dlam = step(rc)
        alpha = 0.99 * min(max_step(s, ds), max_step(lam, dlam))
        alpha = min(alpha, 1.0)
        w += alpha * dw
        nu += alpha * dnu
        s += alpha * ds
        lam += alpha * dlam

    lam_x, lam_a = _to_casadi_duals(n, m, nu, lam, eq_map, in_map)
    best = dict(w=w.copy(), lam_x=lam_x, lam_a=lam_a, iters=it,
                kkt=mpc_qp.kkt_residuals(qp, w, lam_x, lam_a), polished=False)

    if polish:
        act = lam > s
        Ga, ha = G[act], h[act]
        na = Ga.shape[0]
        K = np.zeros((n + me + na, n + me + na))
        K[:n, :n] = H
        K[:n, n:n + me] = E.T
        K[:n, n + me:] = Ga.T
        K[n:n + me, :n] = E
        K[n + me:, :n] = Ga
        rhs = np.concatenate([-g, b, ha])
        try:
            sol = np.linalg.solve(K, rhs)
            wp = sol[:n]
            nup = sol[n:n + me]
            lamp = np.zeros(mi)
            lamp[act] = sol[n + me:]
            ok = (np.all(lamp >= -1e-9) and np.all(G @ wp <= h + 1e-9))
            if ok:
                lamp = np.maximum(lamp, 0)
                lxp, lap = _to_casadi_duals(n, m, nup, lamp, eq_map, in_map)
                kp = mpc_qp.kkt_residuals(qp, wp, lxp, lap)
                if max(kp.values()) <= max(best['kkt'].values()):
                    best = dict(w=wp, lam_x=lxp, lam_a=lap, iters=it, kkt=kp, polished=True)
        except np.linalg.LinAlgError:
            pass
    return best
