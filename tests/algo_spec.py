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
                 repair_top_from=1, repair_top_rep=2, repair_frac=0.5, stable_grow=3,
                 fp32_polish=False, downdate=False, dd_max=24, dd_rebase=False, hook=None,
                 trace=None, fp32_admm=False, border_max=0, weak_base=0.0, border=0,
                 border_extra=4, border_refine=0, light_stable_delta=0):
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
        self.fp32_polish = fp32_polish          # polish preconditioner: the kernel's fp32 sweep inverse
        self.downdate = downdate                # face-adding repairs as downdates of the inverse
        self.dd_max = dd_max                    # ... up to this many added faces per factorization
        self.dd_rebase = dd_rebase              # ... and any repair that keeps the session's base
                                                # faces: the added faces re-downdated from the base
        self.hook = hook                        # (studies) dict filled at the first polish session
        self.trace = trace                      # (studies) list: one event per factorization / repair
        self.fp32_admm = fp32_admm              # (studies) ADMM inverse in fp32 as the kernel's sweep
        self.border = border                    # repairs as the kernel's bordered system on the
                                                # session's base, up to this many columns
        self.border_extra = border_extra        # ... refinement steps past polish_refine (bordered)
        self.border_refine = border_refine      # (study) iterative-refinement steps of W = M U
        self.light_stable_delta = light_stable_delta  # NC <= 128: polish after stable_checks - this
                                                      # (cmpc_wave.hip CMPC_LIGHT_STABLE_DELTA, off)
        self.weak_base = weak_base              # (studies) faces ADMM holds only weakly (gone at
                                                # this fraction of its dual) enter as downdates
        self.border_max = border_max            # (studies) repairs as a bordered system on the
                                                # session's base: up to this many changed faces


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


def sweep_inverse32(H):
    """The kernel's polish inverse in fp32: unit-diagonal scaling, then the symmetric sweep
    (Gauss-Jordan) pivot by pivot in fp32 (the 4-pivot block form keeps the scalar sweep's
    accuracy); M holds -(scaled inverse) until the sign and scaling are undone."""
    H = np.asarray(H, np.float64)
    n = H.shape[0]
    dsc = (1.0 / np.sqrt(np.diag(H))).astype(F32)
    T = (H.astype(F32) * dsc[:, None] * dsc[None, :]).astype(F32)
    for k in range(n):
        piv = T[k, k]
        col = T[:, k].copy()
        col[k] = piv - F32(1)
        T = (T - np.outer(col, col / piv)).astype(F32)
        T[k, k] -= F32(2)
    return (-T * dsc[:, None] * dsc[None, :]).astype(F32)


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

    stats = dict(fact=0, refine=0, dd_faces=0, dd_batches=0, dd_fallback=0, sessions=0,
                 repairs=0, dd_repairs=0)

    def admm_matrix(rho):
        stats['fact'] += 1
        if p.trace is not None:
            p.trace.append(('admm', it_now[0], float(rho)))
        Bt = [B[k][:, [3 * l + a for l in range(4) if stance[k, l] for a in range(3)]] for k in range(N)]
        Rt = np.concatenate([np.tile(p.R[[3 * l + a for a in range(3)]], 1) for k in range(N) for l in range(4) if stance[k, l]]) if nf else np.zeros(0, F32)
        H = condense(A, Bt, p.Q, Rt, p.sigma + rho)
        if p.fp32_admm and nf:
            return ('M', sweep_inverse32(H))
        return np.linalg.cholesky(H.astype(np.float64)).astype(F32) if nf else None

    def solve_L(L, v):
        if isinstance(L, tuple):
            return (L[1] @ v.astype(F32)).astype(F32)
        y = np.linalg.solve(L.astype(np.float64), v.astype(np.float64))
        return np.linalg.solve(L.T.astype(np.float64), y).astype(F32)

    def full(v):
        u = np.zeros(12 * N, F32); u[fidx] = v; return u.reshape(N, 12)

    tri = [(k, l) for k in range(N) for l in range(4) if stance[k, l]]

    def make_basis(code):
        """Reduced basis of the faces in `code` (cmpc_wave.hip polish_setup) and its factorization:
        u = T v + t0; pidx[t] = (px, py, pz) of triple t (-1: no param)."""
        stats['fact'] += 1
        if p.trace is not None:
            p.trace.append(('polish', it_now[0]))
        Bt = []; Rt = []; params = []
        t0 = np.zeros(12 * N, F32)
        pidx = np.full((len(tri), 3), -1, int)
        ti = 0
        for k in range(N):
            cols = []
            for l in range(4):
                if not stance[k, l]:
                    continue
                c = code[ti]
                sx = 1 if c & 2 else (-1 if c & 4 else 0)
                sy = 1 if c & 8 else (-1 if c & 16 else 0)
                zl = bool(c & 1)
                base = 3 * l
                if sx == 0:
                    pidx[ti, 0] = len(params)
                    cols.append(B[k][:, base]); Rt.append(p.R[base]); params.append((k, l, 'x', sx, sy))
                if sy == 0:
                    pidx[ti, 1] = len(params)
                    cols.append(B[k][:, base + 1]); Rt.append(p.R[base + 1]); params.append((k, l, 'y', sx, sy))
                if not zl:
                    pidx[ti, 2] = len(params)
                    col = B[k][:, base + 2] + sx * p.mu * B[k][:, base] + sy * p.mu * B[k][:, base + 1]
                    cols.append(col)
                    Rt.append(p.R[base + 2] + p.mu * p.mu * ((sx != 0) * p.R[base] + (sy != 0) * p.R[base + 1]))
                    params.append((k, l, 'z', sx, sy))
                else:
                    t0[12 * k + base + 2] = p.fz_min
                    t0[12 * k + base] = sx * p.mu * p.fz_min
                    t0[12 * k + base + 1] = sy * p.mu * p.fz_min
                ti += 1
            Bt.append(np.stack(cols, 1).astype(F32) if cols else np.zeros((12, 0), F32))
        H = condense(A, Bt, p.Q, np.array(Rt, F32), p.sigma)
        bs = dict(params=params, t0=t0, pidx=pidx, code=np.array(code).copy(), nr=len(params))
        if p.fp32_polish or p.downdate:
            # an explicit inverse: fp32 as the kernel's sweep computes it, or float64
            bs['M'] = sweep_inverse32(H) if p.fp32_polish else np.linalg.inv(H.astype(np.float64))
            bs['M0'] = bs['M']
        else:
            bs['L'] = np.linalg.cholesky(H.astype(np.float64)).astype(F32)
        return bs

    def apply_inv(bs, r):
        if 'M' in bs:
            return (bs['M'] @ r.astype(bs['M'].dtype)).astype(F32)
        return solve_L(bs['L'], r)

    def expand(bs, v):
        u = bs['t0'].copy()
        for (val, (k, l, ax, sx, sy)) in zip(v, bs['params']):
            b = 12 * k + 3 * l
            if ax == 'x': u[b] = val
            elif ax == 'y': u[b + 1] = val
            else:
                u[b + 2] = val; u[b] += sx * p.mu * val; u[b + 1] += sy * p.mu * val
        return u

    def reduce(bs, g):
        out = np.zeros(bs['nr'], F32)
        for i, (k, l, ax, sx, sy) in enumerate(bs['params']):
            b = 12 * k + 3 * l
            if ax == 'x': out[i] = g[b]
            elif ax == 'y': out[i] = g[b + 1]
            else: out[i] = g[b + 2] + sx * p.mu * g[b] + sy * p.mu * g[b + 1]
        return out

    def v_from(bs, uf):
        return np.array([uf[12 * k + 3 * l + {'x': 0, 'y': 1, 'z': 2}[ax]]
                         for (k, l, ax, sx, sy) in bs['params']], F32)

    def refine(bs, v):
        step = np.inf; prev = np.inf
        for q in range(p.polish_refine + 4):   # cmpc_wave.hip kRefineExtra, kRefineRate
            stats['refine'] += 1
            u = expand(bs, v)
            g, _ = gradient(A, B, d, p.Q, p.R, u.reshape(N, 12))
            dv = apply_inv(bs, reduce(bs, g.reshape(-1)))
            v = v - dv
            step = np.max(np.abs(dv), initial=0)
            if q + 1 >= p.polish_refine and (step <= p.tol_polish * max(1.0, np.max(np.abs(v), initial=0))
                                             or step > 0.5 * prev):
                break
            prev = step
        return v, step

    def check(bs, v, code, step, u_in=None):
        """KKT check of the faces in `code` at v (forces from the basis, cmpc_wave.hip
        polish_check); returns ok, u, the repaired code, loose."""
        u = expand(bs, v) if u_in is None else u_in.astype(F32)
        g, _ = gradient(A, B, d, p.Q, p.R, u.reshape(N, 12))
        g = g.reshape(-1)
        gs = F32(max(np.max(np.abs(g[fidx])), 1e-30))
        us = F32(max(np.max(np.abs(u)), 1.0))
        ok = bool(step <= p.tol_polish * us)
        newcode = np.array(code).copy()
        viol = np.full(len(code), -1.0)
        for ti, (k, l) in enumerate(tri):
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
            vv = max(-lx / gs if sx else 0.0, -ly / gs if sy else 0.0,
                     -l0 / gs if c & 1 else 0.0,
                     0.0 if sx else (abs(fx) - p.mu * fz) / us,
                     0.0 if sy else (abs(fy) - p.mu * fz) / us,
                     0.0 if c & 1 else (p.fz_min - fz) / us)
            viol[ti] = vv
        if p.repair_top > 0 and (len(failed_starts) >= p.repair_top_from or cur_rep[0] >= p.repair_top_rep):
            ncand = int(np.sum(newcode != code))
            kk = max(p.repair_top, int(np.ceil(p.repair_frac * ncand)))
            keep = np.argsort(-viol)[kk:]
            newcode[keep] = np.array(code)[keep]
        loose = bool(step <= p.tol_polish * us) and bool(np.all(viol <= 5.0 * p.tol_polish))
        return ok, u, newcode, loose

    def face_constraints(bs, code_old, code_new):
        """Face additions (code_old -> code_new, no drops) as equalities a'v = c on the basis
        params (cmpc_wave.hip face downdates)."""
        cons = []
        for ti, (k, l) in enumerate(tri):
            add = int(code_new[ti]) & ~int(code_old[ti])
            if not add:
                continue
            px, py, pz = bs['pidx'][ti]
            # fz lock first: a friction face added with it then reads its fz as fz_min
            if add & 1:
                cons.append(({pz: 1.0}, p.fz_min))
            for bit_p, bit_m, pa in ((2, 4, px), (8, 16, py)):
                if add & (bit_p | bit_m):
                    s = 1.0 if add & bit_p else -1.0
                    if pz >= 0:
                        cons.append(({pa: 1.0, pz: -s * float(p.mu)}, 0.0))
                    else:
                        cons.append(({pa: 1.0}, s * float(p.mu) * float(p.fz_min)))
        return cons

    def downdate(bs, v, cons):
        """M <- M - W (A'W)^-1 W' with W = M A, four faces at a time (one panel of the kernel),
        and v projected onto the new equalities in the M metric."""
        M = bs['M']
        for i0 in range(0, len(cons), 4):
            blk = cons[i0:i0 + 4]
            Am = np.zeros((bs['nr'], len(blk)), M.dtype)
            cv = np.zeros(len(blk), M.dtype)
            for j, (a, c) in enumerate(blk):
                for idx, val in a.items():
                    Am[idx, j] = val
                cv[j] = c
            W = (M @ Am).astype(M.dtype)
            S = (Am.T @ W).astype(M.dtype)
            r = (Am.T @ v.astype(M.dtype) - cv).astype(M.dtype)
            v = (v - W @ np.linalg.solve(S.astype(np.float64), r.astype(np.float64)).astype(M.dtype)).astype(F32)
            M = (M - (W @ np.linalg.solve(S.astype(np.float64), W.T.astype(np.float64))).astype(M.dtype)).astype(M.dtype)
            stats['dd_batches'] += 1
        stats['dd_faces'] += len(cons)
        bs = dict(bs); bs['M'] = M
        bs['nadd'] = bs.get('nadd', 0) + len(cons)
        return bs, v

    def border_build(bs, c1):
        """cmpc_wave.hip border_build: the columns of face set c1 against the base bs (new
        parameters for dropped base faces, constraints for added faces), W = M U, S^-1."""
        c0 = bs['code']
        M = bs['M']
        ext, cons = [], []
        for ti, (k, l) in enumerate(tri):
            a, b = int(c0[ti]), int(c1[ti])
            px, py, pz = bs['pidx'][ti]
            sx0 = 1 if a & 2 else (-1 if a & 4 else 0)
            sy0 = 1 if a & 8 else (-1 if a & 16 else 0)
            jz = jx = jy = None
            if (a & 1) and not (b & 1):
                jz = len(ext); ext.append((ti, 2, np.array([sx0 * p.mu, sy0 * p.mu, 1.0], np.float64)))
            if sx0 and not (b & a & 6):
                jx = len(ext); ext.append((ti, 0, np.array([1.0, 0, 0])))
            if sy0 and not (b & a & 24):
                jy = len(ext); ext.append((ti, 1, np.array([0, 1.0, 0])))
            zt = ('v', pz) if not (a & 1) else (('e', jz) if jz is not None else None)
            zc = float(p.fz_min) if (a & 1) else 0.0
            if (b & 1) and not (a & 1):
                cons.append(([('v', pz, 1.0)], float(p.fz_min)))
            for ax, bits in ((0, (b & 6) & ~(a & 6)), (1, (b & 24) & ~(a & 24))):
                if not bits:
                    continue
                sg = 1.0 if bits & (8 if ax else 2) else -1.0
                s0 = sy0 if ax else sx0
                t1 = ('v', py if ax else px) if s0 == 0 else ('e', jy if ax else jx)
                cz = -sg * float(p.mu) if s0 == 0 else 2.0 * s0 * float(p.mu)
                terms = [(t1[0], t1[1], 1.0)] + ([(zt[0], zt[1], cz)] if zt is not None else [])
                cons.append((terms, -cz * zc))
        k = len(ext) + len(cons)
        if k > p.border:
            return None
        nr = bs['nr']
        U = np.zeros((nr, k)); D = np.zeros((k, k))
        Gt = []
        for j, (ti, ax, dvec) in enumerate(ext):
            kk, l = tri[ti]
            u = np.zeros((N, 12), F32); u[kk, 3 * l:3 * l + 3] = dvec
            g, _ = gradient(A, B, np.zeros_like(d), p.Q, p.R, u)
            Gt.append(g.reshape(-1).astype(np.float64))
            U[:, j] = reduce(bs, g.reshape(-1))
        for i, (ti, ax, dvec) in enumerate(ext):
            kk, l = tri[ti]
            for j in range(len(ext)):
                D[i, j] = dvec @ Gt[j][12 * kk + 3 * l:12 * kk + 3 * l + 3]
        for c, (terms, rhs) in enumerate(cons):
            j = len(ext) + c
            for kind, idx, cf in terms:
                if kind == 'v':
                    U[idx, j] += cf
                else:
                    D[idx, j] += cf; D[j, idx] += cf
        Mf = M.astype(np.float64)
        W = Mf @ U
        for _ in range(p.border_refine):  # W += M (U - H0 W), H0 applied through the gradient
            HW = np.zeros_like(W)
            for j in range(k):
                ul = expand(bs, W[:, j].astype(F32)) - bs['t0']
                g, _ = gradient(A, B, np.zeros_like(d), p.Q, p.R, ul.reshape(N, 12))
                HW[:, j] = reduce(bs, g.reshape(-1)) + p.sigma * W[:, j]
            W = W + Mf @ (U - HW)
        S = D - U.T @ W
        stats['bd_cols'] = stats.get('bd_cols', 0) + k
        stats['bd_ext'] = stats.get('bd_ext', 0) + len(ext)
        return dict(ext=ext, cons=cons, W=W, Sinv=np.linalg.inv(S), e=np.zeros(len(ext)), k=k)

    def force_ext(bs, v, bd):
        u = expand(bs, v).astype(np.float64)
        if bd is not None:
            for j, (ti, ax, dvec) in enumerate(bd['ext']):
                kk, l = tri[ti]
                u[12 * kk + 3 * l:12 * kk + 3 * l + 3] += bd['e'][j] * dvec
        return u

    def refine_border(bs, v, bd):
        """refine() with the bordered Newton step (cmpc_wave.hip border_apply)."""
        step = np.inf; prev = np.inf
        M = bs['M'].astype(np.float64)
        for q in range(p.polish_refine + p.border_extra):
            stats['refine'] += 1
            u = force_ext(bs, v, bd)
            g, _ = gradient(A, B, d, p.Q, p.R, u.astype(F32).reshape(N, 12))
            g = g.reshape(-1).astype(np.float64)
            gv = reduce(bs, g.astype(F32)).astype(np.float64)
            b = []
            for j, (ti, ax, dvec) in enumerate(bd['ext']):
                kk, l = tri[ti]
                b.append(dvec @ g[12 * kk + 3 * l:12 * kk + 3 * l + 3])
            for terms, rhs in bd['cons']:
                r = -rhs
                for kind, idx, cf in terms:
                    r += cf * (v[idx] if kind == 'v' else bd['e'][idx])
                b.append(r)
            z = bd['Sinv'] @ (np.array(b) - bd['W'].T @ gv)
            dv = M @ gv - bd['W'] @ z
            ne = len(bd['ext'])
            v = (v - dv).astype(F32)
            bd['e'] = bd['e'] - z[:ne]
            step = max(np.max(np.abs(dv), initial=0), np.max(np.abs(z[:ne]), initial=0))
            if p.trace is not None:
                p.trace.append(('bstep', q, float(step), bd['k'], ne))
            if q + 1 >= p.polish_refine and (step <= p.tol_polish * max(1.0, np.max(np.abs(v), initial=0))
                                             or step > 0.5 * prev):
                break
            prev = step
        return v, step

    def nchanges(c0, c1):
        x = np.array(c0) ^ np.array(c1)
        return int(sum(bin(int(t)).count('1') for t in x))

    def session(zv, code, budget, tried):
        """One polish session from ADMM's face set `code`; returns ok, u, the last repaired code
        and the loose flag."""
        if p.hook is not None and 'code' not in p.hook:
            p.hook.update(code=np.array(code).copy(), rho=rho, z=zv.copy())
        if p.weak_base > 0 and weak_code[0] is not None:
            strong = np.array(code) & weak_code[0]
            bs = make_basis(strong)
            v = v_from(bs, full(zv).reshape(-1))
            cons = face_constraints(bs, strong, code)
            if 0 < len(cons) <= p.dd_max:
                stats['weak_faces'] = stats.get('weak_faces', 0) + len(cons)
                bs, v = downdate(bs, v, cons)
            elif cons:
                stats['fact'] -= 1
                bs = make_basis(code)
                v = v_from(bs, full(zv).reshape(-1))
        else:
            bs = make_basis(code)
            v = v_from(bs, full(zv).reshape(-1))
        rep = 0
        cur_rep[0] = 0
        while True:
            bd = bs.get('bd')
            if bd is not None:
                v, step = refine_border(bs, v, bd)
                ok, u, nc, loose = check(bs, v, code, step, force_ext(bs, v, bd))
            else:
                v, step = refine(bs, v)
                ok, u, nc, loose = check(bs, v, code, step)
            if (not ok and (bs.get('nadd', 0) > 0 or (bd is not None and bd['k'] > 0)) and
                    not step <= p.tol_polish * max(1.0, float(np.max(np.abs(u))))):
                # the downdated preconditioner no longer contracts: refactor the current face set
                stats['dd_fallback'] += 1
                bs = make_basis(code)
                v = v_from(bs, u)
                continue
            if ok:
                return True, u, nc, loose
            if rep >= budget or np.array_equal(nc, code) or nc.tobytes() in tried[:8]:
                return False, u, nc, loose
            tried.append(nc.tobytes())
            rep += 1
            cur_rep[0] = rep
            stats['repairs'] += 1
            drops = np.any((nc & np.array(code)) != np.array(code))
            if p.trace is not None:
                co = np.array(code)
                p.trace.append(('repair', int(np.sum((nc & ~co) != 0)), int(np.sum((co & ~nc) != 0))))
            cons = [] if drops or not p.downdate else face_constraints(bs, code, nc)
            keeps_base = not np.any((nc & bs['code']) != bs['code'])
            bdn = border_build(bs, nc) if p.border > 0 else None
            if bdn is not None:
                stats['dd_repairs'] += 1
                stats['border_repairs'] = stats.get('border_repairs', 0) + 1
                bs = dict(bs); bs['bd'] = bdn
            elif p.border > 0:
                bs = make_basis(nc)
                v = v_from(bs, full(zv).reshape(-1))
            elif p.downdate and not drops and bs.get('nadd', 0) + len(cons) <= p.dd_max:
                stats['dd_repairs'] += 1
                bs, v = downdate(bs, v, cons)
            elif p.border_max > 0 and nchanges(bs['code'], nc) <= p.border_max:
                # (study) the bordered Schur system of the base inverse: the repaired set's exact
                # inverse without a factorization (one symv per changed face)
                stats['border_repairs'] = stats.get('border_repairs', 0) + 1
                b0 = bs['code']
                bs = make_basis(nc)
                stats['fact'] -= 1
                bs['code'] = b0
                v = v_from(bs, u)
            elif p.downdate and p.dd_rebase and keeps_base and \
                    len(face_constraints(bs, bs['code'], nc)) <= p.dd_max:
                # a drop of added faces only: the session's base inverse, downdated afresh
                stats['dd_repairs'] += 1
                stats['dd_rebases'] = stats.get('dd_rebases', 0) + 1
                base = dict(bs); base['M'] = bs['M0']; base['nadd'] = 0
                bs, v = downdate(base, v, face_constraints(bs, bs['code'], nc))
            else:
                bs = make_basis(nc)
                v = v_from(bs, full(zv).reshape(-1))
            code = nc

    cur_rep = [0]  # repairs made so far in the current session (repair_top_rep)
    it_now = [0]   # (studies) the ADMM iteration, for the trace
    weak_code = [None]  # (studies) the face set at a fraction of ADMM's dual (weak_base)

    failed_starts = []
    # the NC >= 128 bins (nf > 96) start from rho / 2 and return to rho after their first
    # failed polish session (cmpc_wave.hip solve_instance, rho_low)
    # the NC <= 128 bins polish one stable iteration earlier (cmpc_wave.hip CMPC_LIGHT_STABLE_DELTA)
    pstable = max(1, p.stable_checks - (p.light_stable_delta if nf <= 128 else 0))
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
        it_now[0] = it
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
        backoff = pstable << min(len(failed_starts), p.backoff_cap)   # cmpc_wave.hip kBackoffCap
        if stable >= pstable * p.stable_grow ** min(len(failed_starts), p.backoff_cap) and it - last_pol >= backoff:
            last_pol = it
            # a session: polish ADMM's face set, then repair it.  A set that started a failed
            # session before is polished once more without repairs; a repair that returns to a
            # set this session already tried ends the session (cmpc_wave.hip kFailMem/kTryMem).
            if p.weak_base > 0:
                _, weak_code[0] = project((xr + F32(1 - p.weak_base) * y / F32(rho)).reshape(-1, 3),
                                          p.mu, p.fz_min)
            start = code.tobytes()
            seen = start in failed_starts[-4:]
            tried = [start]
            stats['sessions'] += 1
            # the ADMM inverse is parked only where a failure restores it (cmpc_wave.hip)
            parked = not rho_low and len(failed_starts) > 0
            budget = 0 if seen else (min(p.repairs, p.late_repairs) if len(failed_starts) >= 2 else p.repairs)
            ok, u, _, loose = session(z, code, budget, tried)
            stable = -backoff  # back off before the next attempt
            if not ok and loose:
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
            elif not parked:
                stats['fact'] += 1  # the polish inverse replaced the ADMM one: refactor
                if p.trace is not None:
                    p.trace.append(('admm-restore', it, float(rho)))
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
    return dict(U=U.reshape(N, 12), status=status, iters=it, nf=nf, **stats)
