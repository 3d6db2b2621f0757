"""Generate the golden fixtures under tests/golden/ (run in the build container).

1. ``ref_inputs.npz`` -- QP *inputs* produced by the reference's own code:
   ``gait.Gait.compute_contact_table`` (gait.py:26-37), ``ComTraj.generate_traj``'s x_ref
   construction (com_trajectory.py:27-104) and ``ComTraj._continuousDynamics`` /
   ``_discreteDynamics`` (com_trajectory.py:221-286), imported from /root/reference with the
   Pinocchio-backed robot model replaced by a synthetic stand-in object (no URDF exists in the
   image; only its outputs m, I_com, foot levers feed the QP).  Pins oracle/mpc_qp.py and
   cmpc/synth.py's discretisation.
2. ``traj_ticks.npz`` -- consecutive MPC ticks of ``ComTraj.generate_traj`` (com_trajectory.py:
   27-207: desired-position clamp, x_ref, contact table, foot levers with touchdown prediction,
   gait.py:21-74) for robots with random gaits (``gait.PHASE_OFFSET`` set per robot), run by the
   reference's own code on a stand-in robot whose base rotation is the full ZYX rotation of its
   state (scipy ``Rotation``).  Inputs are fp32-representable (the C-ABI's boundary type) except
   time and gait, which the C-ABI takes in float64.  Pins oracle/traj_ref.py and
   ``cmpc_generate_traj``.
3. ``leg_ticks.npz`` -- consecutive 1 kHz ticks of the reference's ``LegController.compute_leg_torque``
   for the four legs (leg_controller.py:43-112, with ``Gait.compute_swing_traj_and_touchdown`` /
   ``make_swing_trajectory``, gait.py:77-174) on a stand-in robot that returns given Pinocchio
   quantities (Jacobians, M, C, g, dq, foot states: synthetic, fp32-representable; M SPD).
   Pins oracle/leg_ref.py and ``cmpc_leg_torque``.
4. ``qp_cfg1.npz`` / ``qp_cfg2.npz`` -- synthetic batches (cmpc.synth, SURVEY.md 8(d) configs
   1 and 2) with their KKT-certified float64 optimum from oracle/tight_solver.py, in the
   reference layout (w, lam_x, lam_a) plus the certificate residuals.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))

sys.path.insert(0, str(REPO / "tests"))
from oracle import mpc_qp, tight_solver  # noqa: E402
from parity_util import input_digest  # noqa: E402
from cmpc import synth  # noqa: E402

REF = Path("/root/reference/convex_mpc")


class _Cfg:
    def __init__(self):
        self.base_pos = np.zeros(3)
        self.base_vel = np.zeros(3)


class SyntheticGo2:
    """Stand-in for go2_robot_data.PinGo2Model exposing only what ComTraj.generate_traj reads
    (go2_robot_data.py:171-222, 252-269).  Values are synthetic (no URDF in the image)."""

    def __init__(self, x0=None, m=15.0, I=None, hip=None, feet=None):
        self.current_config = _Cfg()
        self.data = types.SimpleNamespace(Ig=types.SimpleNamespace(
            mass=m, inertia=np.diag([0.11, 0.28, 0.31]) if I is None else I))
        self._x0 = np.zeros(12) if x0 is None else np.asarray(x0, float)
        yaw = self._x0[5]
        c, s = np.cos(yaw), np.sin(yaw)
        self.R_z = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])
        self.R_body_to_world = self.R_z
        self.R_world_to_body = self.R_z.T
        hipxy = synth.HIP_XY if hip is None else hip
        self._hip = {n: np.array([hipxy[i, 0], hipxy[i, 1], 0.0])
                     for i, n in enumerate(("FL", "FR", "RL", "RR"))}
        self._feet = feet
        self.yaw_rate_des_world = 0.0

    def compute_com_x_vec(self):
        return self._x0.reshape(-1, 1).copy()

    def get_hip_offset(self, leg):
        return self._hip[leg]

    def get_foot_lever_world(self):
        return [self._feet[i].copy() for i in range(4)]

    def update_model_simplified(self, q, dq):
        self.current_config.base_pos = np.array(q[0:3], float)
        self.current_config.base_vel = np.array(dq[0:3], float)
        yaw = q[5]
        c, s = np.cos(yaw), np.sin(yaw)
        self.R_z = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])


class SyntheticGo2Full(SyntheticGo2):
    """As SyntheticGo2, but ``R_world_to_body`` is the full base rotation R_z R_y R_x of the
    state's roll/pitch/yaw (what Pinocchio's oMb.rotation is for that state,
    go2_robot_data.py:211-216), computed independently of the oracle with scipy."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        from scipy.spatial.transform import Rotation
        r, p, y = self._x0[3:6]
        R = Rotation.from_euler("ZYX", [y, p, r]).as_matrix()
        self.R_body_to_world = R
        self.R_world_to_body = R.T


def import_reference():
    """Import gait.py / com_trajectory.py from the reference (pure NumPy/SciPy).  Their module
    header imports ``go2_robot_data`` (Pinocchio); that module is replaced by a namespace whose
    PinGo2Model is the synthetic stand-in above."""
    sys.modules["go2_robot_data"] = types.SimpleNamespace(PinGo2Model=SyntheticGo2)
    if not hasattr(np, "trapz"):
        np.trapz = np.trapezoid
    sys.path.insert(0, str(REF))
    import gait  # noqa: F401
    import com_trajectory  # noqa: F401
    return gait, com_trajectory


def make_ref_inputs(n_cases: int = 6):
    gait_mod, ct_mod = import_reference()
    rng = np.random.default_rng(7)
    cases = []
    for c in range(n_cases):
        hz, duty = [(3.0, 0.6), (2.0, 0.5), (3.0, 0.7)][c % 3]
        g = gait_mod.Gait(hz, duty)
        t_now = float(rng.uniform(0, 1.0))
        dt = g.gait_period / 16
        yaw = float(rng.uniform(-np.pi, np.pi))
        x0 = np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), 0.27 + 0.01 * rng.normal(),
                       0.05 * rng.normal(), 0.05 * rng.normal(), yaw,
                       0.3 * rng.normal(), 0.3 * rng.normal(), 0.05 * rng.normal(),
                       0.1 * rng.normal(), 0.1 * rng.normal(), 0.5 * rng.normal()])
        feet = [np.array([synth.HIP_XY[i, 0], synth.HIP_XY[i, 1], -0.27]) + 0.01 * rng.normal(size=3)
                for i in range(4)]
        go2 = SyntheticGo2(x0=x0, feet=feet)
        traj = ct_mod.ComTraj(go2)
        vx, vy, wz = float(rng.uniform(-0.8, 0.8)), float(rng.uniform(-0.4, 0.4)), float(rng.uniform(-2, 2))
        traj.generate_traj(go2, g, t_now, vx, vy, 0.27, wz, time_step=dt)
        N = traj.N
        r_legs = np.stack([traj.r_fl_foot_world, traj.r_fr_foot_world,
                           traj.r_rl_foot_world, traj.r_rr_foot_world], 0).transpose(2, 0, 1)
        cases.append(dict(N=N, dt=dt, hz=hz, duty=duty, t_now=t_now, m=traj.m,
                          I=np.asarray(traj.I_com_world), x0=x0,
                          xref=traj.compute_x_ref_vec(), contact=traj.contact_table,
                          r_legs=r_legs, yaw_avg=np.average(traj.rpy_traj_world[2, :]),
                          Ac=traj.Ac, Bc=traj.Bc, gc=traj.gc,
                          Ad=traj.Ad, Bd=traj.Bd, gd=traj.gd.reshape(-1)))
    out = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{i}_{k}"] = np.asarray(v)
    out["n_cases"] = np.array(n_cases)
    np.savez_compressed(HERE / "ref_inputs.npz", **out)
    print("ref_inputs.npz:", n_cases, "cases")


def _f32(x):
    return np.asarray(np.float32(x), dtype=np.float64)


def make_traj_ticks(n_robots: int = 10, n_ticks: int = 6):
    """Consecutive ticks of the reference's generate_traj, per robot (see module doc)."""
    gait_mod, ct_mod = import_reference()
    rng = np.random.default_rng(11)
    hip = _f32(np.array([[0.1934, 0.0465, 0.0], [0.1934, -0.0465, 0.0],
                         [-0.1934, 0.0465, 0.0], [-0.1934, -0.0465, 0.0]])
               + np.array([[0, 0.0955, 0], [0, -0.0955, 0], [0, 0.0955, 0], [0, -0.0955, 0]]))
    rec = {k: [] for k in ("x0", "pos_des_in", "pos_des_out", "cmd", "t_now", "gait", "N", "dt",
                           "foot_lever", "xref", "contact", "r_feet")}
    for r in range(n_robots):
        hz = [3.0, 2.0, 3.0, 4.0, 2.5][r % 5]
        duty = [0.6, 0.5, 0.75, 0.4, 0.62][r % 5]
        offs = np.array([0.5, 0.0, 0.0, 0.5]) if r % 2 == 0 else rng.uniform(0, 1, 4)
        div = 8 if r == n_robots - 1 else 16          # one N = 8 robot
        g = gait_mod.Gait(hz, duty)
        dt = g.gait_period / div
        t_now = float(rng.uniform(0, 2.0))
        x0 = _f32(np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), 0.27 + 0.01 * rng.normal(),
                            0.05 * rng.normal(), 0.05 * rng.normal(), rng.uniform(-np.pi, np.pi),
                            0.3 * rng.normal(), 0.3 * rng.normal(), 0.05 * rng.normal(),
                            0.1 * rng.normal(), 0.1 * rng.normal(), 0.5 * rng.normal()]))
        go2 = SyntheticGo2Full(x0=x0, feet=[np.zeros(3)] * 4)
        traj = ct_mod.ComTraj(go2)
        # the touchdown prediction reads the hip offsets of ComTraj's dummy model (:139)
        traj.dummy_go2._hip = {n: hip[i].copy() for i, n in enumerate(("FL", "FR", "RL", "RR"))}
        for t in range(n_ticks):
            cmd = _f32([rng.uniform(-0.8, 0.8), rng.uniform(-0.4, 0.4), 0.27 + 0.02 * rng.normal(),
                        rng.uniform(-3, 3)])
            feet = [_f32(hip[i] + np.array([0, 0, -0.27]) + 0.02 * rng.normal(size=3))
                    for i in range(4)]
            go2 = SyntheticGo2Full(x0=x0, feet=feet, hip=hip[:, :2])
            go2._hip = {n: hip[i].copy() for i, n in enumerate(("FL", "FR", "RL", "RR"))}
            gait_mod.PHASE_OFFSET = offs.copy()
            pd_in = np.array(traj.pos_des_world, dtype=np.float64, copy=True)
            traj.generate_traj(go2, g, t_now, cmd[0], cmd[1], cmd[2], cmd[3], time_step=dt)
            assert traj.N == div, (traj.N, div)
            r_feet = np.zeros((16, 4, 3))
            r_feet[:div] = np.stack([traj.r_fl_foot_world, traj.r_fr_foot_world,
                                     traj.r_rl_foot_world, traj.r_rr_foot_world], 0).transpose(2, 0, 1)
            xref = np.zeros((16, 12)); xref[:div] = traj.compute_x_ref_vec().T
            ct = np.zeros((4, 16), np.uint8); ct[:, :div] = traj.contact_table
            for k, v in (("x0", x0), ("pos_des_in", pd_in), ("pos_des_out", traj.pos_des_world),
                         ("cmd", cmd), ("t_now", t_now),
                         ("gait", [g.gait_period, duty, *offs]), ("N", div), ("dt", dt),
                         ("foot_lever", np.stack(feet)), ("xref", xref), ("contact", ct),
                         ("r_feet", r_feet)):
                rec[k].append(np.array(v, copy=True))
            # next tick: time advances one MPC step, the state moves a little
            t_now += dt
            x0 = _f32(x0 + np.concatenate([x0[6:9] * dt, x0[9:12] * dt, 0.05 * rng.normal(size=6)]))
    gait_mod.PHASE_OFFSET = np.array([0.5, 0.0, 0.0, 0.5])
    out = {k: np.stack(v) for k, v in rec.items()}
    out["hip"] = hip
    np.savez_compressed(HERE / "traj_ticks.npz", **out)
    print("traj_ticks.npz:", len(rec["N"]), "ticks")


class LegGo2:
    """Stand-in for PinGo2Model exposing what LegController / Gait's swing planning read
    (go2_robot_data.py:171-173, 271-360): values set per tick by make_leg_ticks."""
    LEGS = ("FL", "FR", "RL", "RR")

    def __init__(self, hip):
        self.current_config = _Cfg()
        self._hip = {n: hip[i].copy() for i, n in enumerate(self.LEGS)}

    def set(self, J_foot, J_full, M, C, g, dq, Jdd, fpos, fvel, body):
        self._Jf, self._Jfull, self._M, self._C, self._g = J_foot, J_full, M, C, g
        self._dq, self._Jdd, self._fp, self._fv = dq, Jdd, fpos, fvel
        self.current_config.base_pos = body[0:3].copy()
        self.current_config.get_dq = lambda: self._dq.copy()
        self.pos_com_world, self.vel_com_world = body[3:6].copy(), body[6:9].copy()
        c, s_ = np.cos(body[9]), np.sin(body[9])
        self.R_z = np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1.0]])
        self.yaw_rate_des_world = body[10]
        self.x_pos_des_world, self.y_pos_des_world = body[11], body[12]
        self.x_vel_des_world, self.y_vel_des_world = body[13], body[14]

    def _i(self, leg):
        return self.LEGS.index(leg)

    def get_hip_offset(self, leg):
        return self._hip[leg]

    def compute_3x3_foot_Jacobian_world(self, leg):
        return self._Jf[self._i(leg)].copy()

    def compute_full_foot_Jacobian_world(self, leg):
        return self._Jfull[self._i(leg)].copy()

    def compute_dynamcis_terms(self):
        return self._g.copy(), self._C.copy(), self._M.copy()

    def get_single_foot_state_in_world(self, leg):
        return self._fp[self._i(leg)].copy(), self._fv[self._i(leg)].copy()

    def compute_Jdot_dq_world(self, leg):
        return self._Jdd[self._i(leg)].copy()


def make_leg_ticks(n_robots: int = 5, n_ticks: int = 150):
    """Consecutive 1 kHz ticks of the reference's leg controller, per robot (see module doc)."""
    gait_mod, _ = import_reference()
    import leg_controller as lc_mod
    rng = np.random.default_rng(13)
    f32 = lambda a: np.asarray(np.float32(a), dtype=np.float64)  # noqa: E731
    hip = f32(np.array([[0.1934, 0.142, 0.0], [0.1934, -0.142, 0.0],
                        [-0.1934, 0.142, 0.0], [-0.1934, -0.142, 0.0]]))
    fixed = {k: [] for k in ("J_foot", "J_full", "M", "C")}
    rec = {k: [] for k in ("robot", "t", "gait", "force", "g", "dq", "Jdot_dq", "foot_pos",
                           "foot_vel", "body", "tau")}
    for r in range(n_robots):
        hz = [5.0, 4.0, 6.0, 5.0, 4.5][r % 5]
        duty = [0.5, 0.6, 0.45, 0.55, 0.5][r % 5]
        offs = np.array([0.5, 0.0, 0.0, 0.5]) if r % 2 == 0 else rng.uniform(0, 1, 4)
        g_ = gait_mod.Gait(hz, duty)
        J_foot = f32(rng.normal(0, 0.2, (4, 3, 3)))
        J_full = f32(rng.normal(0, 0.2, (4, 3, 18)))
        J_full[:, :, 6:] = 0.0
        for l in range(4):
            J_full[l, :, 6 + 3 * l:9 + 3 * l] = J_foot[l]
        Araw = rng.normal(0, 1, (18, 18))
        M = f32(Araw @ Araw.T / 18 + np.diag(rng.uniform(0.05, 1.0, 18)))
        C = f32(rng.normal(0, 0.1, (18, 18)))
        for k, v in (("J_foot", J_foot), ("J_full", J_full), ("M", M), ("C", C)):
            fixed[k].append(v)
        go2 = LegGo2(hip)
        ctrl = lc_mod.LegController()
        t = float(rng.uniform(0, 1.0))
        gait_mod.PHASE_OFFSET = offs.copy()
        yaw = float(rng.uniform(-np.pi, np.pi))
        for _ in range(n_ticks):
            body = f32(np.concatenate([rng.normal(0, 0.5, 2), [0.27 + 0.01 * rng.normal()],
                                       rng.normal(0, 0.5, 2), [0.27 + 0.01 * rng.normal()],
                                       rng.normal(0, 0.3, 3), [yaw], [rng.uniform(-2, 2)],
                                       rng.normal(0, 0.5, 2), rng.uniform(-0.8, 0.8, 2), [0.0]]))
            gv, dq = f32(rng.normal(0, 3, 18)), f32(rng.normal(0, 1, 18))
            Jdd, fpos, fvel = (f32(rng.normal(0, 0.3, (4, 3))) for _ in range(3))
            force = f32(rng.normal(0, 40, 12))
            go2.set(J_foot, J_full, M, C, gv, dq, Jdd, fpos, fvel, body)
            tau = np.zeros(12)
            for l, leg in enumerate(LegGo2.LEGS):
                out = ctrl.compute_leg_torque(leg, go2, g_, force[3 * l:3 * l + 3], t)
                tau[3 * l:3 * l + 3] = out.tau
            for k, v in (("robot", r), ("t", t), ("gait", [g_.gait_period, duty, *offs]),
                         ("force", force), ("g", gv), ("dq", dq), ("Jdot_dq", Jdd),
                         ("foot_pos", fpos), ("foot_vel", fvel), ("body", body), ("tau", tau)):
                rec[k].append(np.array(v, copy=True))
            t += 0.001
            yaw += 0.002
    gait_mod.PHASE_OFFSET = np.array([0.5, 0.0, 0.0, 0.5])
    out = {k: np.stack(v) for k, v in rec.items()}
    for k in ("force", "g", "dq", "Jdot_dq", "foot_pos", "foot_vel", "body"):
        out[k] = out[k].astype(np.float32)       # fp32-representable inputs, stored compactly
    out.update({k: np.stack(v).astype(np.float32) for k, v in fixed.items()})
    out["hip"] = hip.astype(np.float32)
    np.savez_compressed(HERE / "leg_ticks.npz", **out)
    print("leg_ticks.npz:", len(rec["t"]), "ticks")


def make_qp_fixture(cfg: int, B: int, name: str):
    b = synth.make_config(cfg, B=B)
    W, LX, LA, KKT = [], [], [], []
    for i in range(B):
        qp = mpc_qp.build_qp(b['Ad'][i], b['Bd'][i], b['gd'][i], b['x0'][i], b['xref'][i].T,
                             b['contact'][i])
        r = tight_solver.solve(qp)
        k = r['kkt']
        assert max(k.values()) < 1e-8, (i, k)
        W.append(r['w']); LX.append(r['lam_x']); LA.append(r['lam_a'])
        KKT.append([k['stat'], k['prim'], k['comp']])
    np.savez_compressed(HERE / name, cfg=cfg, B=B,
                        Ad=b['Ad'], Bd=b['Bd'], gd=b['gd'], x0=b['x0'], xref=b['xref'],
                        contact=b['contact'], w=np.array(W), lam_x=np.array(LX),
                        lam_a=np.array(LA), kkt=np.array(KKT))
    print(name, B, "instances, max KKT residual", np.max(KKT))


# Instances of the cfg2 benchmark batches (synth.make_batch(65536, seed, mixed=True)) that
# exposed solver weaknesses on the GPU: (seed, index, what happened)
HARD_CASES = [
    (57, 1420, "degenerate vertex: two face sets straddle a weakly active friction face, "
               "neither passed the 1e-5 KKT check in fp32 (status 2 after 1000 iterations)"),
    (24, 30782, "ill-conditioned face set: refinement contracts ~30x per step, 4 steps were "
                "not enough (566 iterations)"),
    (57, 32430, "primal-dual repairs wander between face sets (slowest instance, 273 iterations)"),
    (46, 18051, "slow ADMM, many polish sessions (227 iterations)"),
]


def make_hard_fixture(name: str = "qp_hard.npz"):
    rows = {k: [] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}
    W, LX, LA, KKT = [], [], [], []
    for seed, idx, _ in HARD_CASES:
        b = synth.make_batch(65536, seed=seed, mixed=True)
        for k in rows:
            rows[k].append(b[k][idx])
        qp = mpc_qp.build_qp(b['Ad'][idx], b['Bd'][idx], b['gd'][idx], b['x0'][idx],
                             b['xref'][idx].T, b['contact'][idx])
        r = tight_solver.solve(qp)
        k = r['kkt']
        assert max(k.values()) < 1e-8, (seed, idx, k)
        W.append(r['w']); LX.append(r['lam_x']); LA.append(r['lam_a'])
        KKT.append([k['stat'], k['prim'], k['comp']])
    np.savez_compressed(HERE / name, cases=np.array([[s, i] for s, i, _ in HARD_CASES]),
                        **{k: np.array(v) for k, v in rows.items()}, w=np.array(W),
                        lam_x=np.array(LX), lam_a=np.array(LA), kkt=np.array(KKT))
    print(name, len(W), "instances, max KKT residual", np.max(KKT))


def import_reference_mpc():
    """Import centroidal_mpc.py from the reference with ``casadi`` replaced by the
    conversion-only stand-in (tests/golden/casadi_standin.py; CasADi is not installed) and the
    Pinocchio robot module by the synthetic stand-in, so the reference's QP assembly runs
    unmodified."""
    import_reference()
    sys.path.insert(0, str(HERE))
    import casadi_standin
    sys.modules["casadi"] = casadi_standin
    import centroidal_mpc  # noqa: F401
    return centroidal_mpc


def _traj_standin(Ad, Bd, gd, x0, xref, contact):
    """The ComTraj fields CentroidalMPC reads (centroidal_mpc.py:46, 59-67, 122-285)."""
    N = Bd.shape[0]
    return types.SimpleNamespace(
        N=N, Ad=np.array(Ad, dtype=np.float64), Bd=np.array(Bd, dtype=np.float64),
        gd=np.array(gd, dtype=np.float64).reshape(12, 1),
        initial_x_vec=np.array(x0, dtype=np.float64).reshape(12, 1),
        contact_table=np.array(contact, dtype=np.int32),
        compute_x_ref_vec=lambda: np.array(xref, dtype=np.float64).T.copy())


def make_qp_assembly(name: str = "qp_assembly.npz", n_with_A: int = 16):
    """Golden vectors of the reference's own QP assembly (centroidal_mpc.py:41-67, 122-359) for
    every instance of the qp_cfg1 / qp_cfg2 / qp_hard fixtures, by CentroidalMPC itself:
    ``__init__`` (incl. the structure print of _build_sparse_matrix), then per instance
    ``_update_sparse_matrix`` -> (g, A, lba, uba) and ``_compute_bounds`` -> (lbx, ubx).  A is
    kept (values on its structural pattern, CSC) for the first `n_with_A` instances."""
    import contextlib
    import io
    cm = import_reference_mpc()
    rows = {k: [] for k in ("g", "lba", "uba", "lbx", "ubx", "src")}
    A_vals = []
    pattern = None
    H = None
    printed = None
    k = 0
    for fname in ("qp_cfg1.npz", "qp_cfg2.npz", "qp_hard.npz"):
        fx = np.load(HERE / fname)
        for i in range(fx["w"].shape[0]):
            traj = _traj_standin(fx["Ad"][i], fx["Bd"][i], fx["gd"][i], fx["x0"][i],
                                 fx["xref"][i], fx["contact"][i])
            if printed is None:
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    mpc = cm.CentroidalMPC(None, traj)
                printed = buf.getvalue()
                H = mpc.H_const.full()
            g, A, lb, ub = mpc._update_sparse_matrix(traj)
            lbx, ubx = mpc._compute_bounds(traj)
            if pattern is None:
                pattern = A.sparsity()
            assert np.array_equal(A.sparsity().mask, pattern.mask)
            if k < n_with_A:
                A_vals.append(np.array(A.nonzeros()))
            for key, v in (("g", g), ("lba", lb), ("uba", ub), ("lbx", lbx), ("ubx", ubx)):
                rows[key].append(v.full().reshape(-1))
            rows["src"].append([("qp_cfg1.npz", "qp_cfg2.npz", "qp_hard.npz").index(fname), i])
            k += 1
    colind, row = pattern.csc()
    np.savez_compressed(HERE / name, H=H, A_colind=colind, A_row=row, A_vals=np.array(A_vals),
                        A_shape=np.array(pattern.size()), init_print=np.array(printed),
                        **{key: np.array(v) for key, v in rows.items()})
    print(name, k, "instances;", printed.strip().splitlines()[1:3])


def _certify_one(args):
    Ad, Bd, gd, x0, xref, contact = args
    qp = mpc_qp.build_qp(Ad, Bd, gd, x0, xref.T, contact)
    r = tight_solver.solve(qp)
    k = r["kkt"]
    assert max(k.values()) < 1e-8, k
    return r["w"], r["lam_x"], r["lam_a"], [k["stat"], k["prim"], k["comp"]]


def _certify(batch, idx, procs=8):
    import multiprocessing as mp
    jobs = [tuple(batch[k][i] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")) for i in idx]
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_certify_one, jobs, chunksize=4)
    W, LX, LA, KKT = (np.array(x) for x in zip(*res))
    return W, LX, LA, KKT


def make_cfg3_fixture(name: str = "qp_cfg3.npz", per_bin=(128, 256, 127, 1)):
    """KKT-certified optima of 512 instances of the config-3 batch (synth.make_config(3),
    65,536 trot + mixed), stratified over the solver's free-variable bins NC 96/128/160/192
    (all of the batch's NC = 192 instances).  Inputs are regenerated by the GPU test from the
    deterministic generator (indices + an input digest are stored, not the inputs)."""
    b = synth.make_config(3)
    nf = 3 * (b["contact"] != 0).reshape(b["contact"].shape[0], -1).sum(1)
    bins = np.searchsorted(np.array([96, 128, 160, 192]), nf)
    rng = np.random.default_rng(42)
    idx = np.sort(np.concatenate([rng.choice(np.nonzero(bins == q)[0], min(c, int(np.sum(bins == q))),
                                             replace=False) for q, c in enumerate(per_bin)]))
    W, LX, LA, KKT = _certify(b, idx)
    np.savez_compressed(HERE / name, idx=idx, bins=bins[idx], digest=np.array(input_digest(b, idx)),
                        w=W, lam_x=LX, lam_a=LA, kkt=KKT)
    print(name, len(idx), "instances, per bin", np.bincount(bins[idx], minlength=4),
          "max KKT", KKT.max())


def make_nc192_fixture(name: str = "qp_nc192.npz", want: int = 64):
    """KKT-certified instances of the heaviest bin (more than 160 free forces: > 53 of the 64
    (step, leg) pairs in stance), collected from config-2-distribution batches
    (synth.make_batch(65536, seed, mixed=True), seeds 2000...), inputs stored."""
    rows = {k: [] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}
    seeds = []
    seed = 2000
    while len(seeds) < want:
        b = synth.make_batch(65536, seed=seed, mixed=True)
        nf = 3 * (b["contact"] != 0).reshape(65536, -1).sum(1)
        for i in np.nonzero(nf > 160)[0]:
            if len(seeds) < want:
                for k in rows:
                    rows[k].append(b[k][i])
                seeds.append([seed, i])
        seed += 1
    batch = {k: np.array(v) for k, v in rows.items()}
    W, LX, LA, KKT = _certify(batch, np.arange(want))
    np.savez_compressed(HERE / name, cases=np.array(seeds), **batch, w=W, lam_x=LX, lam_a=LA,
                        kkt=KKT)
    print(name, want, "instances from", seed - 2000, "batches, max KKT", KKT.max())


def _certify_exact_one(args):
    """The certified optimum by oracle/active_set.py, seeded with the NumPy model's answer
    (tests/algo_spec.py; only the seed -- the certificate decides)."""
    from oracle import active_set
    import algo_spec
    Ad, Bd, gd, x0, xref, contact = args
    qp = mpc_qp.build_qp(Ad, Bd, gd, x0, xref.T, contact)
    m = algo_spec.solve(dict(Ad=Ad, Bd=Bd, gd=gd, x0=x0, xref=xref, contact=contact),
                        algo_spec.Params(fp32_polish=True, downdate=True, dd_max=6))
    X = mpc_qp.rollout(Ad, Bd, gd, x0, m["U"].astype(np.float64))
    r = active_set.certified_optimum(qp, np.concatenate([X.reshape(-1), m["U"].reshape(-1)]))
    k = r["kkt"]
    assert max(k.values()) < 1e-8, k
    return r["w"], r["lam_x"], r["lam_a"], [k["stat"], k["prim"], k["comp"]]


NEXT_TICK_NAMED = (1363, 2707, 3458, 3485)


def _one_thread():
    """Pool workers: one BLAS thread each (8 workers x 8 BLAS threads thrash the cores)."""
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def make_next_tick_fixture(name: str = "qp_next_tick.npz", step: int = 4):
    """KKT-certified optima of test_warm_next_tick's batch (config 2 at 4,096, seed 2, x0 moved
    by synth.next_tick): every `step`-th instance (1,024) plus the instances that exposed the
    fp32 KKT check's flat-direction limit in round 4 (3458 cold: fy held at mu fz where the
    optimum is 7.97 N, 1.48e-4; 1363 cold 6.0e-5; 2707 cold 1.34e-4 and 3485 warm 2.11e-4 with
    the light-bin schedule on).  The interior point of oracle/tight_solver.py,
    finished by the exact active-set solve of oracle/active_set.py.  Inputs are regenerated
    from the deterministic generator (indices + digest); U* is stored in fp32 (the test's bar is
    1e-4), the named instances' full (w, lam_x, lam_a) in fp64."""
    import multiprocessing as mp
    b = synth.next_tick(synth.make_config(2, B=4096))
    idx = np.union1d(np.arange(0, 4096, step), np.array(NEXT_TICK_NAMED))
    jobs = [tuple(b[k][i] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")) for i in idx]
    with mp.get_context("fork").Pool(8, initializer=_one_thread) as pool:
        res = pool.map(_certify_exact_one, jobs, chunksize=8)
    W, LX, LA, KKT = (np.array(x) for x in zip(*res))
    named = np.searchsorted(idx, NEXT_TICK_NAMED)
    np.savez_compressed(HERE / name, idx=idx, digest=np.array(input_digest(b, idx)),
                        U=W[:, 12 * 16:].astype(np.float32), kkt=KKT.max(1),
                        named=np.array(NEXT_TICK_NAMED), named_w=W[named], named_lam_x=LX[named],
                        named_lam_a=LA[named])
    print(name, len(idx), "instances, max KKT", KKT.max())


if __name__ == "__main__":
    if len(sys.argv) > 1:  # python tests/golden/make_golden.py make_next_tick_fixture ...
        for fn in sys.argv[1:]:
            globals()[fn]()
        sys.exit(0)
    make_ref_inputs()
    make_traj_ticks()
    make_leg_ticks()
    make_qp_fixture(1, 32, "qp_cfg1.npz")
    make_qp_fixture(2, 64, "qp_cfg2.npz")
    make_hard_fixture()
    make_qp_assembly()
    make_cfg3_fixture()
    make_nc192_fixture()
    make_next_tick_fixture()
