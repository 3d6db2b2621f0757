"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- restatement of the reference's QP data path.

This module restates, in float64 NumPy, how ltinphan/convex-mpc-unitree-go2 turns a robot
state + gait into the contact-force QP that it hands to CasADi/OSQP.  It is the checker for
the HIP path; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The product path never routes through this file.

Every function cites the reference file:line it follows (paths relative to the reference
repo root, ``convex_mpc/``).

Pinning:
  * inputs (contact table, Ac/Bc, Ad/Bd/gd, x_ref) are pinned against golden vectors produced
    by running the reference's own ``gait.py`` / ``com_trajectory.py`` code
    (``tests/golden/make_golden.py``);
  * the QP assembly (H, g, A, lba/uba, lbx/ubx and the init print) is pinned by the
    reference's own ``CentroidalMPC`` (``centroidal_mpc.py:41-67, 122-359``) run unmodified
    under a conversion-only casadi stand-in (``tests/golden/casadi_standin.py``): the golden
    vectors in ``tests/golden/qp_assembly.npz`` (``make_golden.make_qp_assembly``) equal this
    module's ``build_qp`` to 1e-14 on 100 instances (``tests/test_oracle.py``), besides the
    structural invariants the reference prints (H 384x384 nnz 384, A 448x384 nnz 5168 dens
    0.0300).  Only OSQP's own iterate stays unpinnable (CasADi/OSQP are not installed).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.linalg import expm

# --- centroidal_mpc.py:12-17 -------------------------------------------------------------
Q_DIAG = np.array([1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1], dtype=np.float64)
R_DIAG = np.full(12, 1e-5, dtype=np.float64)
MU = 0.8
NX = 12
NU = 12
FZ_MIN = 10.0          # centroidal_mpc.py:127
GRAVITY = 9.81         # com_trajectory.py:268

# --- centroidal_mpc.py:20-36 (OSQP options as passed through CasADi) --------------------
OSQP_OPTS = dict(eps_abs=1e-4, eps_rel=1e-4, max_iter=1000, polish=False,
                 adaptive_rho=True, check_termination=10, adaptive_rho_interval=25,
                 scaling=5, scaled_termination=True, warm_start=True)

# --- gait.py:8 -----------------------------------------------------------------------------
TROT_OFFSETS = np.array([0.5, 0.0, 0.0, 0.5])


def contact_table(t0: float, dt: float, N: int, gait_hz: float = 3.0, duty: float = 0.6,
                  offsets=TROT_OFFSETS) -> np.ndarray:
    """gait.py:26-37 ``Gait.compute_contact_table``: stance mask at mid-step times."""
    period = 1.0 / gait_hz
    t = t0 + np.arange(N) * dt
    t = t + dt / 2
    phases = np.mod(np.asarray(offsets, dtype=np.float64)[:, None] + t[None, :] / period, 1.0)
    return (phases < duty).astype(np.int32)


def skew(v) -> np.ndarray:
    """com_trajectory.py:213-219."""
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=np.float64)


def continuous_dynamics(m: float, I_world: np.ndarray, r_legs: np.ndarray, yaw_avg: float):
    """com_trajectory.py:221-270 ``ComTraj._continuousDynamics``.

    r_legs: (N, 4, 3) foot lever arms COM->foot in world frame per horizon step
    (FL, FR, RL, RR).  Returns Ac (12,12), Bc (N,12,12), gc (12,).
    """
    c, s = np.cos(yaw_avg), np.sin(yaw_avg)
    Rz = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    Ac = np.zeros((12, 12))
    Ac[0:3, 6:9] = np.eye(3)
    Ac[3:6, 9:12] = Rz.T
    N = r_legs.shape[0]
    I_inv = np.linalg.inv(I_world)
    Bc = np.zeros((N, 12, 12))
    for i in range(N):
        for leg in range(4):
            Bc[i, 6:9, 3 * leg:3 * leg + 3] = np.eye(3) / m
            Bc[i, 9:12, 3 * leg:3 * leg + 3] = I_inv @ skew(r_legs[i, leg])
    gc = np.zeros(12)
    gc[8] = -GRAVITY
    return Ac, Bc, gc


def discrete_dynamics(Ac, Bc, gc, dt: float):
    """com_trajectory.py:272-286 ``ComTraj._discreteDynamics``.

    ZOH discretisation (what ``scipy.signal.cont2discrete(method='zoh')`` computes: the
    matrix exponential of [[A, B], [0, 0]] dt) and the 50-point trapezoid of expm(Ac t) gc.
    """
    N = Bc.shape[0]
    Bd = np.zeros((N, 12, 12))
    Ad = None
    for i in range(N):
        M = np.zeros((24, 24))
        M[:12, :12] = Ac
        M[:12, 12:] = Bc[i]
        E = expm(M * dt)
        Ad = E[:12, :12]
        Bd[i] = E[:12, 12:]
    tau = np.linspace(0, dt, 50)
    terms = np.stack([expm(Ac * t) @ gc for t in tau], axis=1)
    gd = np.trapezoid(terms, tau, axis=1)
    return Ad, Bd, gd


def discrete_dynamics_closed_form(Ac, Bc, gc, dt: float):
    """Closed form of :func:`discrete_dynamics` (Ac is nilpotent, Ac @ Ac == 0).

    Ad = I + Ac dt; Bd_k = (I dt + Ac dt^2/2) Bc_k; the 50-point trapezoid of
    (I + Ac t) gc is exact because the integrand is linear in t.
    """
    I = np.eye(12)
    Ad = I + Ac * dt
    S = I * dt + Ac * (dt * dt / 2)
    Bd = np.einsum('ij,kjl->kil', S, Bc)
    gd = S @ gc
    return Ad, Bd, gd


# ------------------------------------------------------------------------------------------
# QP assembly in the reference layout (centroidal_mpc.py:122-359)
# ------------------------------------------------------------------------------------------

def compute_bounds(contact: np.ndarray, fz_min: float = FZ_MIN):
    """centroidal_mpc.py:122-176 ``_compute_bounds`` -> lbx, ubx (384,)."""
    N = contact.shape[1]
    nv = N * (NX + NU)
    lbx = np.full(nv, -np.inf)
    ubx = np.full(nv, np.inf)
    start_u = N * NX
    for k in range(N):
        for leg in range(4):
            base = start_u + 12 * k + 3 * leg
            if contact[leg, k]:
                lbx[base + 2] = max(lbx[base + 2], fz_min)
            else:
                lbx[base:base + 3] = 0.0
                ubx[base:base + 3] = 0.0
    return lbx, ubx


def hessian(N: int, Q=Q_DIAG, R=R_DIAG) -> sp.csc_matrix:
    """centroidal_mpc.py:178-201: H = diag(2Q x N, 2R x N) (zeros skipped)."""
    d = np.concatenate([np.tile(2 * Q, N), np.tile(2 * R, N)])
    return sp.diags(d).tocsc()


def friction_matrix(N: int, mu: float = MU) -> sp.csc_matrix:
    """centroidal_mpc.py:324-359 ``_precompute_friction_matrix`` (4 rows per (k, leg))."""
    rows, cols, vals = [], [], []
    baseU = N * NX
    r0 = 0
    for k in range(N):
        uk0 = baseU + k * NU
        for leg in range(4):
            fx, fy, fz = 3 * leg, 3 * leg + 1, 3 * leg + 2
            for (c, sgn) in ((fx, 1.0), (fx, -1.0), (fy, 1.0), (fy, -1.0)):
                rows += [r0, r0]
                cols += [uk0 + c, uk0 + fz]
                vals += [sgn, -mu]
                r0 += 1
    return sp.csc_matrix((vals, (rows, cols)), shape=(r0, N * (NX + NU)))


def constraint_matrix(Ad: np.ndarray, Bd: np.ndarray, mu: float = MU, structural: bool = True):
    """centroidal_mpc.py:287-321 ``_assemble_A_matrix``: A = [[I + S blkdiag(-Ad), blkdiag(-Bd_k)];
    A_fric].

    The reference builds the dynamics blocks from CasADi SX symbols, so every entry of each
    12x12 block is structurally present.  With ``structural=True`` the returned matrix keeps
    explicit zeros inside the blocks so ``nnz`` matches the reference's 5168.
    """
    N = Bd.shape[0]
    nxN = N * NX
    rows, cols, vals = [], [], []
    # identity on x_{k+1}; combined with the shifted -Ad blocks it is one SX sum, whose
    # sparsity is the union -> the diagonal block rows contain I (12 nnz).
    for i in range(nxN):
        rows.append(i); cols.append(i); vals.append(1.0)
    for k in range(1, N):
        for i in range(NX):
            for j in range(NX):
                rows.append(k * NX + i); cols.append((k - 1) * NX + j); vals.append(-Ad[i, j])
    for k in range(N):
        for i in range(NX):
            for j in range(NU):
                rows.append(k * NX + i); cols.append(nxN + k * NU + j); vals.append(-Bd[k, i, j])
    Aeq = sp.csc_matrix((vals, (rows, cols)), shape=(nxN, N * (NX + NU)))
    if structural:
        # keep explicit zeros (scipy would merge duplicates; entries are unique here)
        pass
    else:
        Aeq.eliminate_zeros()
    Af = friction_matrix(N, mu)
    return sp.vstack([Aeq, Af]).tocsc()


def structural_nnz(N: int = 16) -> int:
    """Structural nnz of the reference A (SX blocks are dense): 12N + 144(N-1) + 144N + 8*4N."""
    return NX * N + NX * NX * (N - 1) + NX * NU * N + 2 * 4 * 4 * N


def linear_cost(xref_cols: np.ndarray, Q=Q_DIAG) -> np.ndarray:
    """centroidal_mpc.py:247-253: g = [vec(-2 Q x_ref) (column-major); 0_{N NU}].

    xref_cols is the reference's (12, N) array (column k = target for x_{k+1}).
    """
    N = xref_cols.shape[1]
    gx = (-2.0 * Q[:, None] * xref_cols).reshape(-1, order='F')
    return np.concatenate([gx, np.zeros(N * NU)])


def constraint_bounds(Ad, gd, x0, contact):
    """centroidal_mpc.py:255-283: lba/uba = [beq; friction l/u]."""
    N = contact.shape[1]
    gd = np.asarray(gd).reshape(-1)
    x0 = np.asarray(x0).reshape(-1)
    beq = np.concatenate([Ad @ x0 + gd, np.tile(gd, N - 1)])
    n_ineq = 16 * N
    l_ineq = np.full(n_ineq, -np.inf)
    u_ineq = np.full(n_ineq, np.inf)
    idx = 0
    for k in range(N):
        for leg in range(4):
            if contact[leg, k] == 1:
                u_ineq[idx:idx + 4] = 0.0
            idx += 4
    return np.concatenate([beq, l_ineq]), np.concatenate([beq, u_ineq])


def build_qp(Ad, Bd, gd, x0, xref_cols, contact, Q=Q_DIAG, R=R_DIAG, mu=MU, fz_min=FZ_MIN):
    """Everything ``CentroidalMPC.solve_QP`` passes to the conic solver
    (centroidal_mpc.py:76-89): h, g, a, lba, uba, lbx, ubx."""
    N = contact.shape[1]
    H = hessian(N, Q, R)
    g = linear_cost(xref_cols, Q)
    A = constraint_matrix(Ad, Bd, mu)
    lba, uba = constraint_bounds(Ad, gd, x0, contact)
    lbx, ubx = compute_bounds(contact, fz_min)
    return dict(h=H, g=g, a=A, lba=lba, uba=uba, lbx=lbx, ubx=ubx, N=N)


def kkt_residuals(qp, w, lam_x, lam_a):
    """KKT residuals of (w, lam_x, lam_a) for the reference QP, CasADi sign convention:

    H w + g + A^T lam_a + lam_x = 0, lam > 0 only where the upper bound is active,
    lam < 0 only where the lower bound is active.
    Returns dict of max-abs residuals (stationarity, primal, dual sign, complementarity).
    """
    H, A = qp['h'], qp['a']
    Aw = A @ w
    stat = H @ w + qp['g'] + A.T @ lam_a + lam_x
    prim = max(np.max(np.maximum(qp['lba'] - Aw, 0)), np.max(np.maximum(Aw - qp['uba'], 0)),
               np.max(np.maximum(qp['lbx'] - w, 0)), np.max(np.maximum(w - qp['ubx'], 0)))

    def comp(lam, v, lo, hi):
        pos = np.maximum(lam, 0)
        neg = np.maximum(-lam, 0)
        with np.errstate(invalid='ignore'):
            cu = np.where(np.isfinite(hi), pos * np.abs(hi - v), pos * np.inf)
            cl = np.where(np.isfinite(lo), neg * np.abs(v - lo), neg * np.inf)
        cu = np.where(pos == 0, 0, cu)
        cl = np.where(neg == 0, 0, cl)
        return float(np.max(np.maximum(cu, cl)))

    return dict(stat=float(np.max(np.abs(stat))), prim=float(prim),
                comp=max(comp(lam_x, w, qp['lbx'], qp['ubx']),
                         comp(lam_a, Aw, qp['lba'], qp['uba'])))


def rollout(Ad, Bd, gd, x0, U):
    """x_{k+1} = Ad x_k + Bd_k u_k + gd (go2_robot_data.py:371-373 / the equality rows)."""
    N = Bd.shape[0]
    X = np.zeros((N, 12))
    x = np.asarray(x0, dtype=np.float64).reshape(-1)
    gd = np.asarray(gd).reshape(-1)
    for k in range(N):
        x = Ad @ x + Bd[k] @ U[k] + gd
        X[k] = x
    return X


def pack_w(X, U) -> np.ndarray:
    """Reference decision layout (centroidal_mpc.py:44, test_MPC.py:190-192):
    w = [vec(X (12,N), 'F'); vec(U (12,N), 'F')] = [x_1..x_N, u_0..u_{N-1}]."""
    return np.concatenate([np.asarray(X).reshape(-1), np.asarray(U).reshape(-1)])


def unpack_w(w, N=16):
    """test_MPC.py:190-192."""
    X = w[:12 * N].reshape((12, N), order='F')
    U = w[12 * N:].reshape((12, N), order='F')
    return X, U
