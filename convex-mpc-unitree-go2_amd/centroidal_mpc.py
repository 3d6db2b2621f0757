"""Drop-in replacement for the reference's ``centroidal_mpc`` module (MI355X solver).

The reference (``convex_mpc/centroidal_mpc.py``) builds a sparse QP each MPC tick and solves it
through CasADi's ``conic('S', 'osqp', ...)``.  This module keeps its public surface --
``CentroidalMPC(go2, traj)``, ``solve_QP(go2, traj, verbose)`` returning ``sol`` with
``sol["x"].full()``, ``sol["lam_x"]``, ``sol["lam_a"]``, ``sol["cost"]``, and the
``solve_time`` / ``update_time`` attributes in ms -- so ``test_MPC.py`` and
``leg_controller.py`` consume it unchanged (``from centroidal_mpc import CentroidalMPC`` with
this directory on ``sys.path``).  The solve runs on the GPU through ``libcmpc.so``
(include/cmpc.h); there is no CPU fallback.

Reference citations: constants ``centroidal_mpc.py:12-38``; class ``:40-120``; bounds
``:122-176``; structure print ``:225-230``; result consumption ``test_MPC.py:184-196``.
"""
from __future__ import annotations

import time

import numpy as np

from cmpc.solver import Plan, SolverParams, STATUS_STRINGS
from cmpc import duals as _duals

# centroidal_mpc.py:12-17
COST_MATRIX_Q = np.diag([1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1])
COST_MATRIX_R = np.diag([1e-5] * 12)
MU = 0.8
NX = 12
NU = 12
FZ_MIN = 10.0  # centroidal_mpc.py:127

# centroidal_mpc.py:20-36 (the reference's OSQP options; eps/max_iter/adaptive interval and
# check_termination map onto cmpc_params, the rest are OSQP-internal and have no counterpart)
OPTS = {
    'warm_start_primal': True,
    'warm_start_dual': True,
    "osqp": {"eps_abs": 1e-4, "eps_rel": 1e-4, "max_iter": 1000, "polish": False,
             "verbose": False, 'adaptive_rho': True, "check_termination": 10,
             'adaptive_rho_interval': 25, "scaling": 5, "scaled_termination": True},
}

SOLVER_NAME: str = "cmpc"


class DM:
    """Minimal stand-in for the CasADi DM results the reference's callers read
    (``sol["x"].full()`` -> (n, 1) float64 array, test_MPC.py:190)."""

    def __init__(self, v):
        self._v = np.asarray(v, dtype=np.float64).reshape(-1, 1)

    def full(self):
        return self._v.copy()

    def __array__(self, dtype=None):
        return self._v if dtype is None else self._v.astype(dtype)

    @property
    def shape(self):
        return self._v.shape


class _SolverHandle:
    """``self.solver`` of the reference exposes ``stats()`` (centroidal_mpc.py:113)."""

    def __init__(self):
        self._stats = {}

    def stats(self):
        return dict(self._stats)


class CentroidalMPC:
    def __init__(self, go2, traj, device=None, params: SolverParams | None = None):
        self.Q = COST_MATRIX_Q
        self.R = COST_MATRIX_R
        self.nvars = traj.N * NX + traj.N * NU
        self.solve_time: float = 0
        self.update_time: float = 0
        self.N = traj.N
        p = params or SolverParams(
            N=traj.N, Q=tuple(np.diag(self.Q)), R=tuple(np.diag(self.R)), mu=MU, fz_min=FZ_MIN,
            eps_abs=OPTS["osqp"]["eps_abs"], eps_rel=OPTS["osqp"]["eps_rel"],
            max_iter=OPTS["osqp"]["max_iter"],
            adaptive_rho_interval=OPTS["osqp"]["adaptive_rho_interval"],
            check_termination=OPTS["osqp"]["check_termination"], max_batch=1)
        self.plan = Plan(p, device=device)
        self.solver = _SolverHandle()
        import torch
        self._torch = torch
        dev = self.plan.device
        N = self.N
        self._buf = dict(
            Ad=torch.empty((1, 12, 12), dtype=torch.float32, device=dev),
            Bd=torch.empty((1, N, 12, 12), dtype=torch.float32, device=dev),
            gd=torch.empty((1, 12), dtype=torch.float32, device=dev),
            x0=torch.empty((1, 12), dtype=torch.float32, device=dev),
            xref=torch.empty((1, N, 12), dtype=torch.float32, device=dev),
            contact=torch.empty((1, 4, N), dtype=torch.uint8, device=dev))
        self._out = (torch.empty((1, 24 * N), dtype=torch.float32, device=dev),
                     torch.empty((1,), dtype=torch.int32, device=dev),
                     torch.empty((1,), dtype=torch.int32, device=dev))
        # the reference's multipliers [lam_x (24N) | lam_a (28N)], kept on the device between
        # ticks for the warm start (cmpc_solve_ref)
        self._lam = torch.empty((1, 52 * N), dtype=torch.float32, device=dev)
        self._warm = False  # no previous solution yet (the reference's x_prev = None)
        self._print_structure()

    def _print_structure(self):
        """centroidal_mpc.py:216-230 (same numbers: H diag 2Q/2R, A = [dynamics; friction]
        with dense 12x12 SX blocks)."""
        N = self.N
        nH = int(np.count_nonzero(np.diag(self.Q))) * N + int(np.count_nonzero(np.diag(self.R))) * N
        nA_rows = N * NX + 16 * N
        nA_nnz = NX * N + NX * NX * (N - 1) + NX * NU * N + 32 * N
        print("\n[QP Init] ===== MPC QP Structure =====")
        print(f"  H: {self.nvars:4d} x {self.nvars:<4d} | nnz = {nH:6d} | dens = {nH / self.nvars ** 2:7.4f}")
        print(f"  A: {nA_rows:4d} x {self.nvars:<4d} | nnz = {nA_nnz:6d} | dens = {nA_nnz / (nA_rows * self.nvars):7.4f}")
        print(f"  vars: {self.nvars:d} | constr: {nA_rows:d} | horizon N = {N}")
        print("[QP Init] ✓ Initialization complete.\n")

    def solve_QP(self, go2, traj, verbose: bool = False):
        torch = self._torch
        t0 = time.perf_counter()
        N = self.N
        Ad = np.asarray(traj.Ad, dtype=np.float64)
        Bd = np.asarray(traj.Bd, dtype=np.float64).reshape(N, NX, NU)
        gd = np.asarray(traj.gd, dtype=np.float64).reshape(NX)
        x0 = np.asarray(traj.initial_x_vec, dtype=np.float64).reshape(NX)
        xref = np.asarray(traj.compute_x_ref_vec(), dtype=np.float64)[:, :N]   # (12, N)
        ct = np.asarray(traj.contact_table)[:, :N]
        host = dict(Ad=Ad[None], Bd=Bd[None], gd=gd[None], x0=x0[None],
                    xref=np.ascontiguousarray(xref.T)[None], contact=(ct != 0)[None])
        for k, v in host.items():
            self._buf[k].copy_(torch.as_tensor(v, dtype=self._buf[k].dtype))
        t1 = time.perf_counter()
        b = self._buf
        # warm start from the previous tick (centroidal_mpc.py:91-95 with OPTS warm_start_primal
        # / warm_start_dual): the previous w and the previous lam_x / lam_a, in place on the
        # device; the multipliers of this solve come back in the reference layout (:108-110)
        kw = {}
        if self._warm and OPTS["warm_start_primal"]:
            kw["w_init"] = self._out[0]
        if self._warm and OPTS["warm_start_dual"]:
            kw["lam_init"] = self._lam
        w, st, it = self.plan.solve(b["Ad"], b["Bd"], b["gd"], b["x0"], b["xref"], b["contact"],
                                    out=self._out, lam_out=self._lam, **kw)
        self._warm = True
        w_np = w.cpu().numpy()[0].astype(np.float64)
        lam = self._lam.cpu().numpy()[0].astype(np.float64)
        status = int(st.cpu().item())
        iters = int(it.cpu().item())
        t2 = time.perf_counter()
        lam_x, lam_a = lam[:24 * N], lam[24 * N:]
        cost = _duals.cost(w_np, xref.T, self.Q, self.R)
        self.update_time = (t1 - t0) * 1e3
        self.solve_time = (t2 - t1) * 1e3
        sol = {"x": DM(w_np), "lam_x": DM(lam_x), "lam_a": DM(lam_a), "cost": DM([cost])}
        # the reference keeps the solution for warm start (centroidal_mpc.py:107-110)
        self.x_prev, self.lam_x_prev, self.lam_a_prev = sol["x"], sol["lam_x"], sol["lam_a"]
        self.solver._stats = {"return_status": STATUS_STRINGS.get(status, str(status)),
                              "iter_count": iters, "success": status in (1, 2)}
        if verbose:
            tc, ts = t1 - t0, t2 - t1
            print(f"[QP SOLVER] update matrix takes {tc*1e3:.3f} ms")
            print(f"[QP SOLVER] solver takes {ts*1e3:.3f} ms")
            print(f"[QP SOLVER] total time = {(tc + ts)*1e3:.3f} ms  ({1.0/(tc + ts):.1f} Hz)")
            print(f"[QP SOLVER] status: {self.solver._stats.get('return_status')}")
        return sol
