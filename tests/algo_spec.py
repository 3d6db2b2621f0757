"""NumPy model of the HIP solver's algorithm (TEST INFRASTRUCTURE).

Mirrors ``convex-mpc-unitree-go2_amd/csrc/cmpc_wave.hip`` step for step (condensed
free-force ADMM with an fp32 preconditioner, accurate error-coordinate gradient, active-set
polish with iterative refinement) so the algorithm's logic can be exercised on CPU.  Not the
oracle: the oracle is ``oracle/tight_solver.py``.
"""
from __future__ import annotations
import numpy as np

F32 = np.float32


class Params:
    def __init__(self, N=16, Q=None, R=None, mu=0.8, fz_min=10.0, rho=1e-4, sigma=1e-6,
                 alpha=1.6, max_iter=400, stable_checks=3, adaptive_interval=25,
                 eps_abs=1e-4, eps_rel=1e-4, polish_refine=4, tol_polish=1e-5, repairs=6,
                 fail_rho=4.0, late_repairs=3, backoff_cap=3, repair_top=2,
                 repair_top_from=1, repair_top_rep=2, repair_frac=0.5, stable_grow=3):
        self.N = N
        self.Q = np.array([1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1], F32) if Q is None else np.asarray(Q, F32)
        self.R = np.full(12, 1e-5, F32) if R is None else np.asarray(R, F32)
        self.mu, self.fz_min = F32(mu), F32(fz_min)
        self.rho, self.sigma, self.alpha = rho, sigma, alpha
        self.max_iter, self.stable_checks = max_iter, stable_checks
        self.adaptive_interval = adaptive_interval
        self.eps_abs, self.eps_rel = eps_abs, eps_rel
        self.polish_refine, self.tol_polish = polish_refine, tol_polish
        self.repairs = repairs
        self.fail_rho, self.late_repairs, self.backoff_cap = fail_rho, late_repairs, backoff_cap
        self.repair_top = repair_top  # >0: a repair changes only the triples of the top violations
        self.repair_top_from = repair_top_from  # ... from the session after this many failed ones
        self.repair_top_rep = repair_top_rep    # ... or from this repair of any session on
        self.repair_frac = repair_frac          # ... at least this fraction of the changed triples
        self.stable_grow = stable_grow          # required face-set stability x this per failed session


def project(v, mu, fz_min):
    """Euclidean projection of each (fx, fy, fz) onto {|fx|<=mu fz, |fy|<=mu fz, fz>=fz_min}.
    Returns (p, code) with code bits: 1 fz at fz_min, 2/4 fx at +/-mu fz, 8/16 fy at +/-."""
    a, b, c = v[..., 0], v[..., 1], v[..., 2]
    A, Bb = np.abs(a), np.abs(b)
    lo, hi = np.minimum(A, Bb), np.maximum(A, Bb)
    z1 = (c + mu * (A + Bb)) / (1 + 2 * mu * mu)
    z2 = (c + mu * hi) / (1 + mu * mu)
    z = np.where(mu * z1 < lo, z1, np.where(mu * z2 < hi, z2, c))
    zl = z < fz_min
    z = np.maximum(z, fz_min)
    lim = mu * z
    x = np.clip(a, -lim, lim)
    y = np.clip(b, -lim, lim)
    code = zl.astype(np.int32)
    code |= np.where(a > lim, 2, 0) | np.where(a < -lim, 4, 0)
    code |= np.where(b > lim, 8, 0) | np.where(b < -lim, 16, 0)
    return np.stack([x, y, z], -1), code


def gradient(A, B, d, Q, R, u):
    """Error-coordinate rollout + adjoint: grad of sum e'Qe + u'Ru (e_{k+1}=Ae_k+B_k u_k+d_k)."""
    N = B.shape[0]
    e = np.zeros(12, F32)
    E = np.zeros((N, 12), F32)
    for k in range(N):
        e = A @ e + (B[k] @ u[k] + d[k])
        E[k] = e
    lam = np.zeros(12, F32)
    g = np.zeros((N, 12), F32)
    for k in range(N - 1, -1, -1):
        lam = 2 * Q * E[k] + A.T @ lam
        g[k] = B[k].T @ lam + 2 * R * u[k]
    return g, E


def condense(A, Bt, Q, Rt, shift):
    """H = 2 Gt' Qbar Gt + diag(2 Rt) + shift I for per-step input matrices Bt[k] (12 x m_k)."""
    N = len(Bt)
    m = [b.shape[1] for b in Bt]
    off = np.concatenate([[0], np.cumsum(m)]).astype(int)
    n = off[-1]
    H = np.zeros((n, n), F32)
    S = np.diag(2 * Q).astype(F32)
    for j in range(N - 1, -1, -1):
        if j < N - 1:
            S = np.diag(2 * Q).astype(F32) + A.T @ S @ A
        W = S @ Bt[j]
        for i in range(j, -1, -1):
            if i < j:
                W = A.T @ W
            blk = Bt[i].T @ W
            H[off[i]:off[i + 1], off[j]:off[j + 1]] = blk
            H[off[j]:off[j + 1], off[i]:off[i + 1]] = blk.T
    H += np.diag(2 * np.asarray(Rt, F32) + F32(shift))
    return H


def solve(inst, p: Params):
    """Solve one instance. inst: dict with Ad, Bd, gd, x0, xref (N,12), contact (4,N)."""
    N = p.N
    A = inst['Ad'].astype(F32); B = inst['Bd'].astype(F32); gd = inst['gd'].astype(F32)
    x0 = inst['x0'].astype(F32); xr = inst['xref'].astype(F32); ct = inst['contact']
    r = np.concatenate([x0[None], xr], 0)
    d = (r[:N] @ A.T + gd - r[1:]).astype(F32)
    stance = ct.T.astype(bool)                                   # (N,4)
    # free variable list (k, leg, axis)
    free = [(k, l, a) for k in range(N) for l in range(4) if stance[k, l] for a in range(3)]
    nf = len(free)
    fidx = np.array([12 * k + 3 * l + a for (k, l, a) in free])

    def admm_matrix(rho):
        Bt = [B[k][:, [3 * l + a for l in range(4) if stance[k, l] for a in range(3)]] for k in range(N)]
        Rt = np.concatenate([np.tile(p.R[[3 * l + a for a in range(3)]], 1) for k in range(N) for l in range(4) if stance[k, l]]) if nf else np.zeros(0, F32)
        H = condense(A, Bt, p.Q, Rt, p.sigma + rho)
        return np.linalg.cholesky(H.astype(np.float64)).astype(F32) if nf else None

    def solve_L(L, v):
        y = np.linalg.solve(L.astype(np.float64), v.astype(np.float64))
        return np.linalg.solve(L.T.astype(np.float64), y).astype(F32)

    def full(v):
        u = np.zeros(12 * N, F32); u[fidx] = v; return u.reshape(N, 12)

    def polish(zv, code):
        # faces per stance triple
        Bt = []; Rt = []; params = []
        t0 = np.zeros(12 * N, F32)
        ti = 0
        for k in range(N):
            cols = []
            for l in range(4):
                if not stance[k, l]:
                    continue
                c = code[ti]; ti += 1
                sx = 1 if c & 2 else (-1 if c & 4 else 0)
                sy = 1 if c & 8 else (-1 if c & 16 else 0)
                zl = bool(c & 1)
                base = 3 * l
                if sx == 0:
                    cols.append(B[k][:, base]); Rt.append(p.R[base]); params.append((k, l, 'x', sx, sy))
                if sy == 0:
                    cols.append(B[k][:, base + 1]); Rt.append(p.R[base + 1]); params.append((k, l, 'y', sx, sy))
                if not zl:
                    col = B[k][:, base + 2] + sx * p.mu * B[k][:, base] + sy * p.mu * B[k][:, base + 1]
                    cols.append(col)
                    Rt.append(p.R[base + 2] + p.mu * p.mu * ((sx != 0) * p.R[base] + (sy != 0) * p.R[base + 1]))
                    params.append((k, l, 'z', sx, sy))
                else:
                    t0[12 * k + base + 2] = p.fz_min
                    t0[12 * k + base] = sx * p.mu * p.fz_min
                    t0[12 * k + base + 1] = sy * p.mu * p.fz_min
            Bt.append(np.stack(cols, 1).astype(F32) if cols else np.zeros((12, 0), F32))
        nr = len(params)
        H = condense(A, Bt, p.Q, np.array(Rt, F32), p.sigma)
        L = np.linalg.cholesky(H.astype(np.float64)).astype(F32)
        zf = full(zv).reshape(-1)

        def expand(v):
            u = t0.copy()
            for (val, (k, l, ax, sx, sy)) in zip(v, params):
                b = 12 * k + 3 * l
                if ax == 'x': u[b] = val
                elif ax == 'y': u[b + 1] = val
                else:
                    u[b + 2] = val; u[b] += sx * p.mu * val; u[b + 1] += sy * p.mu * val
            return u

        def reduce(g):
            out = np.zeros(nr, F32)
            for i, (k, l, ax, sx, sy) in enumerate(params):
                b = 12 * k + 3 * l
                if ax == 'x': out[i] = g[b]
                elif ax == 'y': out[i] = g[b + 1]
                else: out[i] = g[b + 2] + sx * p.mu * g[b] + sy * p.mu * g[b + 1]
            return out

        v = np.array([zf[12 * k + 3 * l + {'x': 0, 'y': 1, 'z': 2}[ax]] for (k, l, ax, sx, sy) in params], F32)
        step = np.inf; prev = np.inf
        for q in range(p.polish_refine + 4):   # cmpc_wave.hip kRefineExtra, kRefineRate
            u = expand(v)
            g, _ = gradient(A, B, d, p.Q, p.R, u.reshape(N, 12))
            dv = solve_L(L, reduce(g.reshape(-1)))
            v = v - dv
            step = np.max(np.abs(dv), initial=0)
            if q + 1 >= p.polish_refine and (step <= p.tol_polish * max(1.0, np.max(np.abs(v), initial=0))
                                             or step > 0.5 * prev):
                break
            prev = step
        u = expand(v)
        g, _ = gradient(A, B, d, p.Q, p.R, u.reshape(N, 12))
        g = g.reshape(-1)
        gs = F32(max(np.max(np.abs(g[fidx])), 1e-30))
        us = F32(max(np.max(np.abs(u)), 1.0))
        ok = bool(step <= p.tol_polish * us)
        newcode = code.copy()
        viol = np.full(len(code), -1.0)
        ti = 0
        for k in range(N):
            for l in range(4):
                if not stance[k, l]:
                    continue
                c = code[ti]
                b = 12 * k + 3 * l
                sx = 1 if c & 2 else (-1 if c & 4 else 0)
                sy = 1 if c & 8 else (-1 if c & 16 else 0)
                fx, fy, fz = u[b:b + 3]
                lx = -sx * g[b] if sx else 0.0
                ly = -sy * g[b + 1] if sy else 0.0
                l0 = g[b + 2] - p.mu * (lx + ly)
                tol_d = p.tol_polish * gs
                tol_p = p.tol_polish * us
                nc = c
                if sx and lx < -tol_d: ok = False; nc &= ~6
                if sy and ly < -tol_d: ok = False; nc &= ~24
                if (c & 1) and l0 < -tol_d: ok = False; nc &= ~1
                if not sx and abs(fx) > p.mu * fz + tol_p: ok = False; nc |= (2 if fx > 0 else 4)
                if not sy and abs(fy) > p.mu * fz + tol_p: ok = False; nc |= (8 if fy > 0 else 16)
                if not (c & 1) and fz < p.fz_min - tol_p: ok = False; nc |= 1
                newcode[ti] = nc
                # largest relative violation (cmpc_wave.hip polish_check `viol`)
                v = max(-lx / gs if sx else 0.0, -ly / gs if sy else 0.0,
                        -l0 / gs if c & 1 else 0.0,
                        0.0 if sx else (abs(fx) - p.mu * fz) / us,
                        0.0 if sy else (abs(fy) - p.mu * fz) / us,
                        0.0 if c & 1 else (p.fz_min - fz) / us)
                viol[ti] = v
                ti += 1
        if p.repair_top > 0 and (len(failed_starts) >= p.repair_top_from or cur_rep[0] >= p.repair_top_rep):
            ncand = int(np.sum(newcode != code))
            kk = max(p.repair_top, int(np.ceil(p.repair_frac * ncand)))
            keep = np.argsort(-viol)[kk:]
            newcode[keep] = code[keep]
        self_newcode[0] = newcode
        self_loose[0] = bool(step <= p.tol_polish * us) and bool(np.all(viol <= 5.0 * p.tol_polish))
        return ok, u

    self_newcode = [None]
    cur_rep = [0]  # repairs made so far in the current session (repair_top_rep)
    self_loose = [False]

    failed_starts = []
    # the NC >= 128 bins (nf > 96) start from rho / 2 and return to rho after their first
    # failed polish session (cmpc_wave.hip solve_instance, rho_low)
    rho_low = nf > 96
    rho = p.rho * (0.5 if rho_low else 1.0)
    L = admm_matrix(rho)
    x = np.zeros(nf, F32); z = np.zeros(nf, F32); y = np.zeros(nf, F32)
    g0, _ = gradient(A, B, d, p.Q, p.R, full(x))
    g0 = g0.reshape(-1)[fidx]               # = q of the condensed QP (gradient at 0)
    nq = float(np.max(np.abs(g0), initial=0.0))
    prev_code = None; stable = 0; last_pol = 0
    status = -2; it = 0; U = None
    for it in range(1, p.max_iter + 1):
        g, _ = gradient(A, B, d, p.Q, p.R, full(x))
        g = g.reshape(-1)[fidx]
        rhs = F32(rho) * (z - x) - g - y
        xt = x + solve_L(L, rhs)
        xr = F32(p.alpha) * xt + F32(1 - p.alpha) * z
        x = F32(p.alpha) * xt + F32(1 - p.alpha) * x
        zn, code = project((xr + y / F32(rho)).reshape(-1, 3), p.mu, p.fz_min)
        zn = zn.reshape(-1)
        y = y + F32(rho) * (xr - zn)
        z = zn
        if prev_code is not None and np.array_equal(code, prev_code):
            stable += 1
        else:
            stable = 0
        prev_code = code
        backoff = p.stable_checks << min(len(failed_starts), p.backoff_cap)   # cmpc_wave.hip kBackoffCap
        if stable >= p.stable_checks * p.stable_grow ** min(len(failed_starts), p.backoff_cap) and it - last_pol >= backoff:
            last_pol = it
            # a session: polish ADMM's face set, then repair it.  A set that started a failed
            # session before is polished once more without repairs; a repair that returns to a
            # set this session already tried ends the session (cmpc_wave.hip kFailMem/kTryMem).
            start = code.tobytes()
            seen = start in failed_starts[-4:]
            tried = [start]
            cur_rep[0] = 0
            ok, u = polish(z, code)
            rep = 0
            budget = 0 if seen else (min(p.repairs, p.late_repairs) if len(failed_starts) >= 2 else p.repairs)
            while not ok and rep < budget:   # cmpc_wave.hip kLateRepairs
                c2 = self_newcode[0]
                if np.array_equal(c2, code) or c2.tobytes() in tried[:8]:
                    break
                code = c2
                tried.append(code.tobytes())
                rep += 1
                cur_rep[0] = rep
                ok, u = polish(z, code)
            stable = -backoff  # back off before the next attempt
            if not ok and self_loose[0]:
                ok = True  # the session ends within the loose tolerance (kLooseTol): accepted
            if ok:
                status = 1; U = u; break
            if not seen:
                failed_starts.append(start)
            if len(failed_starts) == 1 and not seen:
                # the first failed session: continue at 4 x rho0 (cmpc_wave.hip kFailRho)
                rho_low = False; rho = p.fail_rho * p.rho; L = admm_matrix(rho)
            elif rho_low:
                rho_low = False; rho = p.rho; L = admm_matrix(rho)
        if p.adaptive_interval and it % p.adaptive_interval == 0:
            rp = np.max(np.abs(x - z)); rd = np.max(np.abs(g + y))
            npn = max(np.max(np.abs(x)), np.max(np.abs(z)), 1e-30)
            # OSQP normalisation max(|P x|, |q|, |y|), with |P x| <= |g| + |q| approximated
            nd = max(np.max(np.abs(g)), nq, np.max(np.abs(y)), 1e-30)
            nr = rho * np.sqrt((rp / npn) / (rd / nd + 1e-30))
            nr = min(max(nr, 1e-6), 1e6)
            if nr > 5 * rho or nr < rho / 5:
                rho = nr; L = admm_matrix(rho); rho_low = False
    if U is None:
        U = full(z).reshape(-1)
    return dict(U=U.reshape(N, 12), status=status, iters=it, nf=nf)
