"""Synthetic Go2 trot QP batches.

The reference builds one QP per MPC tick from a Pinocchio model of the Go2
(``com_trajectory.py:27-211``).  No URDF exists in this image, so batches are drawn from the
distribution SURVEY.md section 8(d) fixes: random yaw / command velocity / state per
instance, the reference's x_ref construction (``com_trajectory.py:78-104``), the trot contact
table (``gait.py:26-37``), foot levers planted in the world and zeroed in swing
(``com_trajectory.py:142,159``), and the closed-form ZOH discretisation of
``com_trajectory.py:221-286`` (Ac is nilpotent, so Ad = I + Ac dt, Bd_k = (I dt + Ac dt^2/2)
Bc_k, gd = (I dt + Ac dt^2/2) gc exactly).

All arrays are float64, row-major, in the boundary layout of ``include/cmpc.h``:
  Ad (B,12,12), Bd (B,N,12,12), gd (B,12), x0 (B,12), xref (B,N,12), contact (B,4,N) uint8.
"""
from __future__ import annotations

import numpy as np

N_HORIZON = 16
GAIT_HZ = 3.0
GAIT_DUTY = 0.6
DT = (1.0 / GAIT_HZ) / 16          # test_MPC.py:67  MPC_DT = GAIT_T / 16
MASS = 15.0                        # synthetic Go2 composite mass [kg]
INERTIA_BODY = np.diag([0.11, 0.28, 0.31])   # synthetic composite inertia about COM [kg m^2]
HIP_XY = np.array([[0.1934, 0.142], [0.1934, -0.142], [-0.1934, 0.142], [-0.1934, -0.142]])
Z_DES = 0.27                       # test_MPC.py:57
GRAVITY = 9.81
TROT_OFFSETS = np.array([0.5, 0.0, 0.0, 0.5])   # gait.py:8


def _rz(yaw):
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.zeros(np.shape(yaw) + (3, 3))
    R[..., 0, 0] = c; R[..., 0, 1] = -s
    R[..., 1, 0] = s; R[..., 1, 1] = c
    R[..., 2, 2] = 1.0
    return R


def contact_table(t0, dt, N, gait_hz=GAIT_HZ, duty=GAIT_DUTY, offsets=TROT_OFFSETS):
    """gait.py:26-37, batched over leading dims of ``t0``/``duty``/``offsets``.

    Returns (..., 4, N) uint8 (1 = stance)."""
    t0 = np.asarray(t0, dtype=np.float64)
    t = t0[..., None] + np.arange(N) * dt + dt / 2                      # (..., N)
    offs = np.asarray(offsets, dtype=np.float64)
    ph = np.mod(offs[..., :, None] + t[..., None, :] / (1.0 / gait_hz), 1.0)  # (..., 4, N)
    return (ph < np.asarray(duty)[..., None, None]).astype(np.uint8)


def skew_batch(r):
    """com_trajectory.py:213-219 on (..., 3) -> (..., 3, 3)."""
    S = np.zeros(r.shape[:-1] + (3, 3))
    S[..., 0, 1] = -r[..., 2]; S[..., 0, 2] = r[..., 1]
    S[..., 1, 0] = r[..., 2];  S[..., 1, 2] = -r[..., 0]
    S[..., 2, 0] = -r[..., 1]; S[..., 2, 1] = r[..., 0]
    return S


def discretize(m, I_world, r_legs, yaw_avg, dt):
    """com_trajectory.py:221-286 in closed form, batched.

    m (B,), I_world (B,3,3), r_legs (B,N,4,3), yaw_avg (B,) -> Ad (B,12,12),
    Bd (B,N,12,12), gd (B,12)."""
    B, N = r_legs.shape[:2]
    Rz = _rz(yaw_avg)
    Ac = np.zeros((B, 12, 12))
    Ac[:, 0:3, 6:9] = np.eye(3)
    Ac[:, 3:6, 9:12] = np.swapaxes(Rz, -1, -2)
    Iinv = np.linalg.inv(I_world)
    Bc = np.zeros((B, N, 12, 12))
    for leg in range(4):
        Bc[:, :, 6:9, 3 * leg:3 * leg + 3] = np.eye(3) / m[:, None, None, None]
        Bc[:, :, 9:12, 3 * leg:3 * leg + 3] = np.einsum('bij,bnjk->bnik', Iinv,
                                                       skew_batch(r_legs[:, :, leg]))
    S = np.eye(12)[None] * dt + Ac * (dt * dt / 2)
    Ad = np.eye(12)[None] + Ac * dt
    Bd = np.einsum('bij,bnjk->bnik', S, Bc)
    gc = np.zeros(12); gc[8] = -GRAVITY
    gd = np.einsum('bij,j->bi', S, gc)
    return Ad, Bd, gd


def make_batch(B: int, seed: int, mixed: bool = False, N: int = N_HORIZON, dt: float = DT,
               t0=None):
    """Draw ``B`` independent QP instances.

    mixed=False: config 1 (shared trot table at t0, default 0).
    mixed=True : config 2 (per-instance phase offsets U(0,1)^4, duty U(0.4,0.8), at least
                 one stance foot per step).
    Returns a dict of float64/uint8 arrays plus the raw generation parameters.
    """
    rng = np.random.default_rng(seed)
    yaw = rng.uniform(-np.pi, np.pi, B)
    vx = rng.uniform(-0.8, 0.8, B)
    vy = rng.uniform(-0.4, 0.4, B)
    wz = rng.uniform(-4.0, 4.0, B)
    Rz = _rz(yaw)
    v_des = np.einsum('bij,bj->bi', Rz, np.stack([vx, vy, np.zeros(B)], -1))

    x0 = np.zeros((B, 12))
    x0[:, 0:2] = rng.uniform(-1, 1, (B, 2))
    x0[:, 2] = rng.normal(0.27, 0.01, B)
    x0[:, 3:5] = rng.normal(0, 0.05, (B, 2))
    x0[:, 5] = yaw
    x0[:, 6:9] = v_des + rng.normal(0, 0.1, (B, 3))
    x0[:, 9:11] = rng.normal(0, 0.2, (B, 2))
    x0[:, 11] = wz

    # x_ref (com_trajectory.py:47-104): clamped desired position + v t, yaw + wz t
    t_vec = (np.arange(N) + 1) * dt
    pos_des = np.concatenate([x0[:, 0:2] + rng.uniform(-0.1, 0.1, (B, 2)),
                              np.full((B, 1), Z_DES)], axis=1)
    xref = np.zeros((B, N, 12))
    xref[:, :, 0:3] = pos_des[:, None, :] + v_des[:, None, :] * t_vec[None, :, None]
    xref[:, :, 5] = yaw[:, None] + wz[:, None] * t_vec[None, :]
    xref[:, :, 6:9] = v_des[:, None, :]
    xref[:, :, 11] = wz[:, None]

    if mixed:
        offs = rng.uniform(0, 1, (B, 4))
        duty = rng.uniform(0.4, 0.8, B)
        ct = contact_table(np.zeros(B), dt, N, duty=duty, offsets=offs)
        none = ct.sum(axis=1) == 0                       # (B, N) columns with no stance foot
        if np.any(none):
            bi, ki = np.nonzero(none)
            legs = rng.integers(0, 4, bi.shape[0])
            ct[bi, legs, ki] = 1
    else:
        t0v = 0.0 if t0 is None else t0
        ct = np.broadcast_to(contact_table(np.asarray(t0v), dt, N), (B, 4, N)).copy()

    # foot levers: planted foot in world, lever = foot - com(t); zero in swing
    foot_z = -Z_DES + rng.normal(0, 0.01, (B, 4))
    hip_w = np.einsum('bij,lj->bli', Rz[:, :2, :2], HIP_XY)          # (B,4,2)
    r0 = np.concatenate([hip_w, foot_z[..., None]], axis=-1)        # (B,4,3)
    drift = v_des[:, None, :] * (t_vec - dt)[None, :, None]         # (B,N,3)
    r_legs = r0[:, None, :, :] - drift[:, :, None, :]
    r_legs = r_legs * ct.transpose(0, 2, 1)[..., None]

    m = np.full(B, MASS)
    I_world = np.einsum('bij,jk,blk->bil', Rz, INERTIA_BODY, Rz)
    yaw_avg = xref[:, :, 5].mean(axis=1)
    Ad, Bd, gd = discretize(m, I_world, r_legs, yaw_avg, dt)
    return dict(Ad=Ad, Bd=Bd, gd=gd, x0=x0, xref=xref, contact=ct,
                m=m, I_world=I_world, r_legs=r_legs, yaw_avg=yaw_avg, dt=dt, N=N)


HIP_OFFSETS = np.concatenate([HIP_XY, np.zeros((4, 1))], axis=1)   # body frame, legs FL FR RL RR


def make_tick_inputs(B: int, seed: int, mixed: bool = False, N: int = N_HORIZON,
                     gait_hz: float = GAIT_HZ):
    """Per-robot inputs of one MPC tick before ``ComTraj.generate_traj`` (com_trajectory.py:27-35):
    the state, the persistent desired position, the command, the time, the gait and the current
    foot levers -- what ``cmpc_generate_traj`` consumes (include/cmpc.h).  Same state / command
    distribution as :func:`make_batch`; mixed=True draws per-robot phase offsets U(0,1)^4 and
    duty U(0.4,0.8).  fp32-representable where the boundary is fp32."""
    rng = np.random.default_rng(seed)
    f32 = lambda a: np.asarray(a, np.float32).astype(np.float64)   # noqa: E731
    yaw = rng.uniform(-np.pi, np.pi, B)
    vx, vy, wz = rng.uniform(-0.8, 0.8, B), rng.uniform(-0.4, 0.4, B), rng.uniform(-4.0, 4.0, B)
    Rz = _rz(yaw)
    v_des = np.einsum('bij,bj->bi', Rz, np.stack([vx, vy, np.zeros(B)], -1))
    x0 = np.zeros((B, 12))
    x0[:, 0:2] = rng.uniform(-1, 1, (B, 2))
    x0[:, 2] = rng.normal(0.27, 0.01, B)
    x0[:, 3:5] = rng.normal(0, 0.05, (B, 2))
    x0[:, 5] = yaw
    x0[:, 6:9] = v_des + rng.normal(0, 0.1, (B, 3))
    x0[:, 9:11] = rng.normal(0, 0.2, (B, 2))
    x0[:, 11] = wz
    x0 = f32(x0)
    pos_des = x0[:, 0:3] + np.concatenate([rng.uniform(-0.15, 0.15, (B, 2)),
                                           np.zeros((B, 1))], axis=1)
    cmd = f32(np.stack([vx, vy, np.full(B, Z_DES), wz], -1))
    period = 1.0 / gait_hz
    if mixed:
        gait = np.concatenate([np.full((B, 1), period), rng.uniform(0.4, 0.8, (B, 1)),
                               rng.uniform(0, 1, (B, 4))], axis=1)
    else:
        gait = np.tile(np.array([period, GAIT_DUTY, *TROT_OFFSETS]), (B, 1))
    t_now = rng.uniform(0.0, 10.0, B)
    hip_w = np.einsum('bij,lj->bli', Rz[:, :2, :2], HIP_XY)
    foot_lever = f32(np.concatenate([hip_w, (-Z_DES + rng.normal(0, 0.01, (B, 4)))[..., None]], -1))
    m = np.full(B, MASS)
    I_world = np.einsum('bij,jk,blk->bil', Rz, INERTIA_BODY, Rz)
    return dict(x0=x0, pos_des=pos_des, cmd=cmd, t_now=t_now, gait=gait, foot_lever=foot_lever,
                hip=f32(HIP_OFFSETS), m=m, I_world=I_world, dt=period / N, N=N)


CONFIGS = {
    0: dict(B=1, seed=0, mixed=False),
    1: dict(B=256, seed=1, mixed=False),
    2: dict(B=4096, seed=2, mixed=True),
}


def next_tick(batch: dict, seed: int = 5) -> dict:
    """The next MPC tick's problem in the warm-start proxy (tests, bench, certify_sample): the
    state x0 moves by N(0, 2e-3) on position / attitude and N(0, 2e-2) on the velocities; the
    reference, gait and dynamics stay (centroidal_mpc.py:91-95 warm-starts such a tick from the
    previous solution)."""
    rng = np.random.default_rng(seed)
    out = dict(batch)
    out["x0"] = batch["x0"] + rng.normal(scale=[2e-3] * 6 + [2e-2] * 6, size=batch["x0"].shape)
    return out


def make_config(cfg: int, B: int | None = None):
    if cfg == 3:
        Bt = 65536 if B is None else B
        a = make_batch((Bt + 1) // 2, 3, mixed=False)
        b = make_batch(Bt // 2, 1003, mixed=True)
        out = {}
        for k in ('Ad', 'Bd', 'gd', 'x0', 'xref', 'contact', 'm', 'I_world', 'r_legs', 'yaw_avg'):
            out[k] = np.empty((Bt,) + a[k].shape[1:], dtype=a[k].dtype)
            out[k][0::2] = a[k]
            out[k][1::2] = b[k]
        out['dt'] = a['dt']; out['N'] = a['N']
        return out
    c = dict(CONFIGS[cfg])
    if B is not None:
        c['B'] = B
    return make_batch(**c)
