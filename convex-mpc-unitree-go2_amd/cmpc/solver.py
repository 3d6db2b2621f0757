"""Batched solver on device tensors: the C-ABI wrapped for PyTorch-ROCm buffers.

``Plan`` mirrors what ``CentroidalMPC.__init__`` builds once (``centroidal_mpc.py:41-67``:
constants, sparsity, solver object); ``Plan.solve`` is the batched equivalent of
``solve_QP``'s update + solve (``centroidal_mpc.py:69-120``).  PyTorch is used only for device
memory and streams.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field, fields
from typing import Optional

import torch

from . import _lib

STATUS_STRINGS = {1: "solved", 2: "solved inaccurate", -2: "maximum iterations reached",
                  -10: "unsolved"}


@dataclass
class SolverParams:
    """cmpc_params (include/cmpc.h).  Defaults = the reference's constants
    (centroidal_mpc.py:12-38, :127) plus this solver's ADMM/polish settings."""
    N: int = 16
    Q: tuple = (1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1)
    R: tuple = (1e-5,) * 12
    mu: float = 0.8
    fz_min: float = 10.0
    eps_abs: float = 1e-4
    eps_rel: float = 1e-4
    max_iter: int = 1000
    rho: float = 1e-4
    sigma: float = 1e-6
    alpha: float = 1.6
    adaptive_rho_interval: int = 25
    polish_stable: int = 3
    polish_refine: int = 2
    polish_tol: float = 1e-5
    polish_repairs: int = 6
    check_termination: int = 1   # OPTS check_termination (reference: 10; include/cmpc.h)
    max_batch: int = 65536

    def to_c(self) -> _lib.CParams:
        c = _lib.CParams()
        c.abi_version = _lib.ABI_VERSION
        for f in fields(self):
            val = getattr(self, f.name)
            if f.name in ("Q", "R"):
                if len(val) != 12:
                    raise ValueError(f"{f.name} must have 12 entries")
                setattr(c, f.name, (ctypes.c_float * 12)(*[float(v) for v in val]))
            else:
                setattr(c, f.name, val)
        return c


class CmpcError(RuntimeError):
    pass


def _check(lib, rc: int, what: str):
    if rc != _lib.CMPC_OK:
        raise CmpcError(f"{what} failed ({rc}): {_lib.last_error(lib)}")


def _dev_tensor(t: torch.Tensor, name: str, dtype, shape) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a device (cuda/ROCm) tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


class Plan:
    """Owns a cmpc_plan (device workspace for up to params.max_batch instances)."""

    def __init__(self, params: Optional[SolverParams] = None, device=None):
        self.params = params or SolverParams()
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise CmpcError("cmpc: no ROCm device available (the solver has no CPU fallback)")
        dv = torch.device("cuda") if device is None else torch.device(device)
        if dv.type != "cuda":
            raise ValueError(f"cmpc: plan device must be a ROCm (cuda) device, got {dv}")
        self.device = torch.device("cuda", torch.cuda.current_device() if dv.index is None
                                   else dv.index)
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            cp = self.params.to_c()
            d = _lib.CParams()
            self.lib.cmpc_params_default(ctypes.byref(d))
            if d.abi_version != _lib.ABI_VERSION:
                if d.abi_version not in _lib.ABI_COMPAT:
                    raise CmpcError(f"cmpc: library ABI {d.abi_version}, this binding is ABI "
                                    f"{_lib.ABI_VERSION} (an ABI-5 A/B build loads with "
                                    f"CMPC_ALLOW_ABI5=1)")
                cp.abi_version = d.abi_version   # (A/B experiments only: same layout and kernels)
            _check(self.lib, self.lib.cmpc_plan_create(ctypes.byref(cp), ctypes.byref(h)),
                   "cmpc_plan_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.cmpc_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _same_device(self, t: torch.Tensor):
        """The plan's workspace and streams live on self.device: every tensor must too."""
        if t.device != self.device:
            raise ValueError(f"cmpc: tensors are on {t.device} but the plan was created on "
                             f"{self.device}")

    def set_timing(self, enable: bool):
        _check(self.lib, self.lib.cmpc_plan_set_timing(self._h, int(bool(enable))),
               "cmpc_plan_set_timing")

    def set_team(self, max_batch: int):
        """Small-batch (team) mode for solves of B <= max_batch: four waves per QP.
        -1 = automatic (B <= 4 x CUs, the default), 0 = off (cmpc_plan_set_team)."""
        _check(self.lib, self.lib.cmpc_plan_set_team(self._h, int(max_batch)),
               "cmpc_plan_set_team")

    def team_batch(self) -> int:
        """The largest batch solved in team mode (cmpc_plan_team_batch)."""
        v = ctypes.c_int64()
        _check(self.lib, self.lib.cmpc_plan_team_batch(self._h, ctypes.byref(v)),
               "cmpc_plan_team_batch")
        return int(v.value)

    def set_heavy_first(self, min_batch: int):
        """Submit the NC 144 / 160 register class first for solves of B >= min_batch: -1 =
        automatic (B > 16 x CUs, the default), 0 = never (cmpc_plan_set_heavy_first)."""
        _check(self.lib, self.lib.cmpc_plan_set_heavy_first(self._h, int(min_batch)),
               "cmpc_plan_set_heavy_first")

    def heavy_first_batch(self) -> int:
        """The smallest batch that submits the NC 144 / 160 class first, 0 = never
        (cmpc_plan_heavy_first_batch)."""
        v = ctypes.c_int64()
        _check(self.lib, self.lib.cmpc_plan_heavy_first_batch(self._h, ctypes.byref(v)),
               "cmpc_plan_heavy_first_batch")
        return int(v.value)

    def solve_kernels(self, B: int) -> list:
        """Names of the solve kernels a batch of B launches, per timing slot (None: slot not
        launched), as cmpc_plan_solve_kernel reports them."""
        if not hasattr(self.lib, "cmpc_plan_solve_kernel"):  # (older A/B builds)
            return [None] * _lib.NUM_SOLVE_KERNELS
        out = []
        for k in range(_lib.NUM_SOLVE_KERNELS):
            r = self.lib.cmpc_plan_solve_kernel(self._h, int(B), k)
            out.append(r.decode() if r else None)
        return out

    def stats(self, reset: bool = False) -> dict:
        """Acceptance statistics since plan creation or the last reset (cmpc_plan_stats):
        loose acceptances and the answers returned as status 2 by the certified bound or a
        stalled downdated refinement.  Synchronises the device."""
        keys = ("loose", "status2_cert", "guard_refactors", "reserved")
        if not hasattr(self.lib, "cmpc_plan_stats"):  # (ABI-5 A/B builds)
            return {k: None for k in keys[:3]}
        v = (ctypes.c_uint64 * _lib.NUM_STATS)()
        _check(self.lib, self.lib.cmpc_plan_stats(self._h, v, int(bool(reset))), "cmpc_plan_stats")
        return {k: int(x) for k, x in zip(keys[:3], list(v))}

    def timing_read(self):
        """-> (ms_per_kernel, calls_per_kernel) of the solve kernels since the last read, one
        entry per timing slot (_lib.KERNEL_BINS: 0 = NC 128 + 96, 1 = NC 160 + 144, 2 = NC 192)."""
        ms = (ctypes.c_float * 4)()       # room for the round-1 ABI's four slots (A/B builds)
        calls = (ctypes.c_int32 * 4)()
        _check(self.lib, self.lib.cmpc_plan_timing_read(self._h, ms, calls),
               "cmpc_plan_timing_read")
        k = _lib.NUM_SOLVE_KERNELS
        return list(ms)[:k], list(calls)[:k]

    def solve(self, Ad, Bd, gd, x0, xref, contact, out=None, stream=None, w_init=None,
              y_init=None, y_out=None, lam_init=None, lam_out=None):
        """Solve B instances; all inputs are device tensors (layouts: include/cmpc.h).

        Returns (w (B, 24N) fp32, status (B,) int32, iters (B,) int32).  Asynchronous on
        ``stream`` (default: torch's current stream).

        Warm start (cmpc_solve_warm; the reference's x0 / lam_x0 warm start,
        centroidal_mpc.py:91-95): ``w_init`` (B, 24N) a previous w, ``y_init`` (B, 12N) a
        previous dual.  ``y_out`` (B, 12N) receives the dual at the returned forces; pass
        ``y_out=True`` to allocate it, in which case the return is (w, status, iters, y).

        Reference multipliers (cmpc_solve_ref; centroidal_mpc.py:91-95, 108-110):
        ``lam_init`` (B, 52N) warm duals [lam_x | lam_a] in CasADi's layout and convention,
        ``lam_out`` (B, 52N) the multipliers of the returned point (``lam_out=True``
        allocates it; the return is then (w, status, iters, lam)).  Not combinable with
        y_init / y_out."""
        N = self.params.N
        B = Ad.shape[0]
        f32 = torch.float32
        _dev_tensor(Ad, "Ad", f32, (B, 12, 12))
        _dev_tensor(Bd, "Bd", f32, (B, N, 12, 12))
        _dev_tensor(gd, "gd", f32, (B, 12))
        _dev_tensor(x0, "x0", f32, (B, 12))
        _dev_tensor(xref, "xref", f32, (B, N, 12))
        _dev_tensor(contact, "contact", torch.uint8, (B, 4, N))
        self._same_device(Ad)
        for t in (Bd, gd, x0, xref, contact):
            if t.device != Ad.device:
                raise ValueError("all inputs must be on the same device")
        if out is None:
            w = torch.empty((B, 24 * N), dtype=f32, device=Ad.device)
            status = torch.empty((B,), dtype=torch.int32, device=Ad.device)
            iters = torch.empty((B,), dtype=torch.int32, device=Ad.device)
        else:
            w, status, iters = out
            _dev_tensor(w, "w", f32, (B, 24 * N))
            _dev_tensor(status, "status", torch.int32, (B,))
            _dev_tensor(iters, "iters", torch.int32, (B,))
        if stream is None:
            stream = torch.cuda.current_stream(Ad.device)
        sp = ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
        if lam_init is not None or lam_out is not None:
            if y_init is not None or y_out is not None:
                raise ValueError("lam_init/lam_out (reference layout) and y_init/y_out "
                                 "(cmpc layout) are exclusive")
            ret_l = lam_out is True
            if ret_l:
                lam_out = torch.empty((B, 52 * N), dtype=f32, device=Ad.device)
            for t, name, shape in ((w_init, "w_init", (B, 24 * N)), (lam_init, "lam_init", (B, 52 * N)),
                                   (lam_out, "lam_out", (B, 52 * N))):
                if t is not None:
                    _dev_tensor(t, name, f32, shape)
                    self._same_device(t)
            pt = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else None)  # noqa: E731
            with torch.cuda.device(Ad.device):
                rc = self.lib.cmpc_solve_ref(
                    self._h, ctypes.c_int64(B),
                    *[pt(t) for t in (Ad, Bd, gd, x0, xref, contact, w_init, lam_init, w, lam_out,
                                      status, iters)], sp)
            _check(self.lib, rc, "cmpc_solve_ref")
            return (w, status, iters, lam_out) if ret_l else (w, status, iters)
        ret_y = y_out is True
        if ret_y:
            y_out = torch.empty((B, 12 * N), dtype=f32, device=Ad.device)
        if w_init is None and y_init is None and y_out is None:
            with torch.cuda.device(Ad.device):
                rc = self.lib.cmpc_solve(self._h, ctypes.c_int64(B),
                                         *[ctypes.c_void_p(t.data_ptr()) for t in
                                           (Ad, Bd, gd, x0, xref, contact, w, status, iters)], sp)
            _check(self.lib, rc, "cmpc_solve")
            return w, status, iters
        for t, name, shape in ((w_init, "w_init", (B, 24 * N)), (y_init, "y_init", (B, 12 * N)),
                               (y_out, "y_out", (B, 12 * N))):
            if t is not None:
                _dev_tensor(t, name, f32, shape)
                if t.device != Ad.device:
                    raise ValueError("all inputs must be on the same device")

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr() if t is not None else None)
        with torch.cuda.device(Ad.device):
            rc = self.lib.cmpc_solve_warm(
                self._h, ctypes.c_int64(B),
                *[ptr(t) for t in (Ad, Bd, gd, x0, xref, contact, w_init, y_init, w, y_out,
                                   status, iters)], sp)
        _check(self.lib, rc, "cmpc_solve_warm")
        if ret_y:
            return w, status, iters, y_out
        return w, status, iters

    def build_dynamics(self, mass, inertia, r_feet, xref, dt, out=None, stream=None):
        """Discrete dynamics (Ad, Bd, gd) of B robots on the device -- the reference's
        ComTraj._continuousDynamics + _discreteDynamics (com_trajectory.py:221-286) in closed
        form.  mass (B,), inertia (B,3,3) I_com_world, r_feet (B,N,4,3) COM->foot lever arms
        (legs FL FR RL RR), xref (B,N,12) as for solve(); all fp32 device tensors."""
        N = self.params.N
        B = mass.shape[0]
        f32 = torch.float32
        _dev_tensor(mass, "mass", f32, (B,))
        _dev_tensor(inertia, "inertia", f32, (B, 3, 3))
        _dev_tensor(r_feet, "r_feet", f32, (B, N, 4, 3))
        _dev_tensor(xref, "xref", f32, (B, N, 12))
        self._same_device(mass)
        for t in (inertia, r_feet, xref):
            if t.device != mass.device:
                raise ValueError("all inputs must be on the same device")
        if out is None:
            Ad = torch.empty((B, 12, 12), dtype=f32, device=mass.device)
            Bd = torch.empty((B, N, 12, 12), dtype=f32, device=mass.device)
            gd = torch.empty((B, 12), dtype=f32, device=mass.device)
        else:
            Ad, Bd, gd = out
            _dev_tensor(Ad, "Ad", f32, (B, 12, 12))
            _dev_tensor(Bd, "Bd", f32, (B, N, 12, 12))
            _dev_tensor(gd, "gd", f32, (B, 12))
        if stream is None:
            stream = torch.cuda.current_stream(mass.device)
        sp = ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
        with torch.cuda.device(mass.device):
            rc = self.lib.cmpc_build_dynamics(
                self._h, ctypes.c_int64(B), ctypes.c_float(dt),
                *[ctypes.c_void_p(t.data_ptr()) for t in (mass, inertia, r_feet, xref, Ad, Bd, gd)],
                sp)
        _check(self.lib, rc, "cmpc_build_dynamics")
        return Ad, Bd, gd


    def generate_traj(self, x0, pos_des, cmd, t_now, gait, foot_lever, hip, dt, out=None,
                      stream=None):
        """Reference trajectory, contact table and foot levers of B robots on the device -- the
        reference's ComTraj.generate_traj (com_trajectory.py:27-207) up to the dynamics
        (cmpc_generate_traj, include/cmpc.h).  x0 (B,12) fp32; pos_des (B,3) fp64, updated in
        place (ComTraj.pos_des_world); cmd (B,4) fp32 [vx_body, vy_body, z_des, yaw_rate];
        t_now (B,) fp64; gait (B,6) fp64 [period, duty, 4 phase offsets]; foot_lever (B,4,3)
        fp32; hip (4,3) fp32.  Returns (xref (B,N,12), contact (B,4,N) uint8,
        r_feet (B,N,4,3))."""
        N = self.params.N
        B = x0.shape[0]
        f32, f64 = torch.float32, torch.float64
        _dev_tensor(x0, "x0", f32, (B, 12))
        _dev_tensor(pos_des, "pos_des", f64, (B, 3))
        _dev_tensor(cmd, "cmd", f32, (B, 4))
        _dev_tensor(t_now, "t_now", f64, (B,))
        _dev_tensor(gait, "gait", f64, (B, 6))
        _dev_tensor(foot_lever, "foot_lever", f32, (B, 4, 3))
        _dev_tensor(hip, "hip", f32, (4, 3))
        self._same_device(x0)
        for t in (pos_des, cmd, t_now, gait, foot_lever, hip):
            if t.device != x0.device:
                raise ValueError("all inputs must be on the same device")
        if out is None:
            xref = torch.empty((B, N, 12), dtype=f32, device=x0.device)
            contact = torch.empty((B, 4, N), dtype=torch.uint8, device=x0.device)
            r_feet = torch.empty((B, N, 4, 3), dtype=f32, device=x0.device)
        else:
            xref, contact, r_feet = out
            _dev_tensor(xref, "xref", f32, (B, N, 12))
            _dev_tensor(contact, "contact", torch.uint8, (B, 4, N))
            _dev_tensor(r_feet, "r_feet", f32, (B, N, 4, 3))
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        sp = ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
        with torch.cuda.device(x0.device):
            rc = self.lib.cmpc_generate_traj(
                self._h, ctypes.c_int64(B), ctypes.c_double(dt),
                *[ctypes.c_void_p(t.data_ptr()) for t in (x0, pos_des, cmd, t_now, gait,
                                                          foot_lever, hip, xref, contact, r_feet)],
                sp)
        _check(self.lib, rc, "cmpc_generate_traj")
        return xref, contact, r_feet


    def leg_torque(self, t, gait, force, J_foot, J_full, M, C, g, dq, Jdot_dq, foot_pos, foot_vel,
                   body, hip, state, tau_max=45.0, out=None, stream=None):
        """The reference's leg controller tick for B robots (cmpc_leg_torque, include/cmpc.h;
        leg_controller.py:43-112 + the clip of test_MPC.py:227-228).  ``force`` is (B, 12) fp32
        or a (B, >=12) fp32 view whose rows start at U[:, 0] (e.g. w[:, 12N:]); everything else
        fp64 device tensors; ``state`` (B, 4, 8) is updated in place (initialise with
        :func:`leg_state`).  Returns tau (B, 12) fp64."""
        B = t.shape[0]
        f64 = torch.float64
        _dev_tensor(t, "t", f64, (B,))
        _dev_tensor(gait, "gait", f64, (B, 6))
        if (not isinstance(force, torch.Tensor) or force.device.type != "cuda" or
                force.dtype != torch.float32 or force.dim() != 2 or force.shape[0] != B or
                force.shape[1] < 12 or force.stride(1) != 1):
            raise ValueError("force must be a (B, >=12) fp32 device tensor with unit column stride")
        for name, x, shp in (("J_foot", J_foot, (B, 4, 3, 3)), ("J_full", J_full, (B, 4, 3, 18)),
                             ("M", M, (B, 18, 18)), ("C", C, (B, 18, 18)), ("g", g, (B, 18)),
                             ("dq", dq, (B, 18)), ("Jdot_dq", Jdot_dq, (B, 4, 3)),
                             ("foot_pos", foot_pos, (B, 4, 3)), ("foot_vel", foot_vel, (B, 4, 3)),
                             ("body", body, (B, 16)), ("hip", hip, (4, 3)),
                             ("state", state, (B, 4, 8))):
            _dev_tensor(x, name, f64, shp)
        for x in (t, gait, force, J_foot, J_full, M, C, g, dq, Jdot_dq, foot_pos, foot_vel, body,
                  hip, state):
            self._same_device(x)
        tau = torch.empty((B, 12), dtype=f64, device=t.device) if out is None else out
        _dev_tensor(tau, "tau", f64, (B, 12))
        if stream is None:
            stream = torch.cuda.current_stream(t.device)
        sp = ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
        P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        with torch.cuda.device(t.device):
            rc = self.lib.cmpc_leg_torque(
                self._h, ctypes.c_int64(B), P(t), P(gait), P(force),
                ctypes.c_int64(force.stride(0)), *[P(x) for x in (J_foot, J_full, M, C, g, dq,
                                                               Jdot_dq, foot_pos, foot_vel, body,
                                                               hip, state)],
                ctypes.c_double(tau_max), P(tau), sp)
        _check(self.lib, rc, "cmpc_leg_torque")
        return tau


def leg_state(B: int, device="cuda") -> torch.Tensor:
    """Fresh leg-controller memory for cmpc_leg_torque: last mask 2 (LegController.__init__,
    leg_controller.py:40-41), everything else 0."""
    s = torch.zeros((B, 4, 8), dtype=torch.float64, device=device)
    s[:, :, 0] = 2.0
    return s


def to_device_batch(batch: dict, device="cuda") -> dict:
    """float64/uint8 numpy batch (cmpc.synth layout) -> contiguous device tensors."""
    out = {}
    for k in ("Ad", "Bd", "gd", "x0", "xref"):
        out[k] = torch.as_tensor(batch[k], dtype=torch.float32).contiguous().to(device)
    out["contact"] = torch.as_tensor(batch["contact"], dtype=torch.uint8).contiguous().to(device)
    return out


def solve_batch(batch: dict, params: Optional[SolverParams] = None, plan: Optional[Plan] = None):
    """Convenience: numpy batch in, (w, status, iters) numpy out (synchronises)."""
    plan = plan or Plan(params)
    d = to_device_batch(batch, plan.device)
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize(plan.device)
    return w.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
