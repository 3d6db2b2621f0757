"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- fast KKT-certified optimum of the reference QP,
seeded by a candidate answer.

``tight_solver.solve`` reaches the certified optimum of ``centroidal_mpc.py``'s QP from
scratch (interior point + polish, ~3 s per instance).  Certifying a whole batch of the HIP
path's answers (every instance of a 65,536 batch) needs something faster, and the candidate
already names the face set: this module guesses the active set from the candidate's tight rows,
solves the equality-constrained KKT system of the reference layout exactly (float64, the same
system ``tight_solver``'s polish solves), and repeats primal-dual active-set steps (drop rows
with a negative multiplier, add violated rows) until the KKT conditions hold.  The result is
accepted only with the same certificate as the golden fixtures: ``mpc_qp.kkt_residuals`` of
the reference-assembled QP (stationarity, primal feasibility, complementarity) within
``CERT_TOL``; otherwise it falls back to ``tight_solver.solve``.  The QP is strictly convex
(H diagonal positive, ``centroidal_mpc.py:178-201``), so a certified point IS the unique
optimum whatever the seed was; the seed only decides how fast it is found.

Layout and multiplier convention as ``tight_solver`` (CasADi: H w + g + A' lam_a + lam_x = 0).
"""
from __future__ import annotations

import numpy as np

from . import mpc_qp, tight_solver

CERT_TOL = 1e-8


def _kkt_solve(H, g, E, b, G, h, act):
    n, me = H.shape[0], E.shape[0]
    Ga, ha = G[act], h[act]
    na = Ga.shape[0]
    K = np.zeros((n + me + na, n + me + na))
    K[:n, :n] = H
    K[:n, n:n + me] = E.T
    K[:n, n + me:] = Ga.T
    K[n:n + me, :n] = E
    K[n + me:, :n] = Ga
    sol = np.linalg.solve(K, np.concatenate([-g, b, ha]))
    lam = np.zeros(G.shape[0])
    lam[act] = sol[n + me:]
    return sol[:n], sol[n:n + me], lam


def certified_optimum(qp, w_seed, tight: float = 1e-5, max_steps: int = 30):
    """The certified optimum of ``qp`` (dict as ``mpc_qp.build_qp``), found from the candidate
    ``w_seed`` (384,).  Returns dict(w, lam_x, lam_a, kkt, steps, fallback); the caller checks
    the certificate (max kkt <= CERT_TOL: it fails only if the seed's active-set steps cycle
    AND the interior point diverges)."""
    H = qp['h'].toarray()
    g = qp['g']
    E, b, eq_map, G, h, in_map = tight_solver._split_constraints(qp)
    n, m = H.shape[0], qp['a'].shape[0]
    w_seed = np.asarray(w_seed, np.float64)
    scale = max(1.0, float(np.max(np.abs(w_seed[12 * qp['N']:]))))
    act = (G @ w_seed - h) >= -tight * scale   # the candidate's faces (rows it holds tight)
    seen = set()
    fallback_ok = max_steps > 0   # (a negative max_steps: no fallback, |max_steps| steps)
    for step in range(abs(max_steps)):
        key = act.tobytes()
        if key in seen:   # the active-set steps cycle: certify from scratch
            break
        seen.add(key)
        try:
            w, nu, lam = _kkt_solve(H, g, E, b, G, h, act)
        except np.linalg.LinAlgError:
            break
        viol = (G @ w - h) > 1e-10 * scale
        neg = act & (lam < 0.0)
        if not viol.any() and not neg.any():
            lam_x, lam_a = tight_solver._to_casadi_duals(n, m, nu, np.maximum(lam, 0.0), eq_map,
                                                         in_map)
            kkt = mpc_qp.kkt_residuals(qp, w, lam_x, lam_a)
            if max(kkt.values()) <= CERT_TOL:
                return dict(w=w, lam_x=lam_x, lam_a=lam_a, kkt=kkt, steps=step, fallback=False)
            break
        act = (act & ~neg) | viol
    if not fallback_ok:
        return dict(w=w_seed, lam_x=None, lam_a=None, kkt=dict(stat=np.inf), steps=-1,
                    fallback=True)
    # from scratch: the interior point, finished by the active-set steps from its faces (its
    # unpolished point can sit ~5e-7 off in directions only R weighs); a failed interior point
    # (it diverges on rare instances) is returned as is and fails the certificate
    r = tight_solver.solve(qp)
    if max(r['kkt'].values()) <= CERT_TOL and max_steps > 0:
        r2 = certified_optimum(qp, r['w'], tight=tight, max_steps=-max_steps)
        if not r2['fallback']:
            r = r2
    return dict(w=r['w'], lam_x=r['lam_x'], lam_a=r['lam_a'], kkt=r['kkt'], steps=-1,
                fallback=True)


def certify_batch_item(batch, i, w_seed):
    """Certified optimum of instance ``i`` of a synthetic batch (keys Ad, Bd, gd, x0, xref
    (B, N, 12), contact (B, 4, N)), seeded by ``w_seed``."""
    qp = mpc_qp.build_qp(batch['Ad'][i], batch['Bd'][i], batch['gd'][i], batch['x0'][i],
                         batch['xref'][i].T, batch['contact'][i])
    return certified_optimum(qp, w_seed)
