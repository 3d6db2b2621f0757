"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- batched restatement of the reference's per-tick
reference-trajectory / contact-schedule / foot-lever generation.

Restates, in float64 NumPy, ``ComTraj.generate_traj`` (``convex_mpc/com_trajectory.py:27-207``)
for a batch of robots, with the Pinocchio model replaced by the few quantities the reference
reads from it:
  * ``go2.compute_com_x_vec()`` -> x0 (12,)                      (com_trajectory.py:37)
  * ``go2.R_z`` = R_z(x0[5]), ``go2.R_world_to_body`` = (R_z R_y R_x)(rpy)'  (go2_robot_data.py:
    211-222; the base rotation of the floating base whose ZYX angles are x0[3:6])
  * ``go2.get_foot_lever_world()`` -> foot_lever (4, 3)        (:113, go2_robot_data.py:261-269)
  * ``go2.get_hip_offset(leg)`` -> hip (4, 3), body frame      (gait.py:46, go2_robot_data.py:171-173)
  * ``dummy_go2.update_model_simplified(q, dq)`` only sets base_pos = q[0:3],
    base_vel = dq[0:3] (body-frame velocity) and R_z = R_z(q[5])  (go2_robot_data.py:224-250)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this file; the
product path never does.  Pinned against ``tests/golden/traj_ticks.npz``, produced by the
reference's own ``ComTraj.generate_traj`` + ``Gait`` (tests/golden/make_golden.py).

Batched layouts (the C-ABI's, include/cmpc.h ``cmpc_generate_traj``):
  x0 (B,12); pos_des (B,3) float64 state; cmd (B,4) = [vx_body, vy_body, z_des, yaw_rate];
  t_now (B,) float64; gait (B,6) float64 = [period, duty, offset FL, FR, RL, RR];
  foot_lever (B,4,3); hip (4,3)
  -> pos_des' (B,3), xref (B,N,12), contact (B,4,N) uint8, r_feet (B,N,4,3).
"""
from __future__ import annotations

import numpy as np

MAX_POS_ERROR = 0.1      # com_trajectory.py:47
TD_HEIGHT = 0.02         # gait.py:57 (pos_norminal_term z)


def rot_zyx(rpy):
    """(...,3) roll, pitch, yaw -> (...,3,3) R = R_z(yaw) R_y(pitch) R_x(roll) (body -> world),
    the rotation whose Pinocchio ``matrixToRpy`` is rpy (go2_robot_data.py:74-93, 211-216)."""
    r, p, y = rpy[..., 0], rpy[..., 1], rpy[..., 2]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    R = np.empty(rpy.shape[:-1] + (3, 3))
    R[..., 0, 0] = cy * cp
    R[..., 0, 1] = cy * sp * sr - sy * cr
    R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp
    R[..., 1, 1] = sy * sp * sr + cy * cr
    R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp
    R[..., 2, 1] = cp * sr
    R[..., 2, 2] = cp * cr
    return R


def rz(yaw):
    """go2_robot_data.py:218-222 (R_z of the yaw)."""
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.zeros(np.shape(yaw) + (3, 3))
    R[..., 0, 0] = c; R[..., 0, 1] = -s
    R[..., 1, 0] = s; R[..., 1, 1] = c
    R[..., 2, 2] = 1.0
    return R


def phase_mask(t, period, duty, offsets):
    """gait.py:26-37 core: stance = mod(offset + t / period, 1) < duty.
    t (B,K), period/duty (B,), offsets (B,4) -> (B,4,K) bool."""
    ph = np.mod(offsets[:, :, None] + t[:, None, :] / period[:, None, None], 1.0)
    return ph < duty[:, None, None]


def generate_traj(x0, pos_des, cmd, t_now, gait, foot_lever, hip, dt, N):
    """com_trajectory.py:27-207 ``ComTraj.generate_traj`` (reference/contact/lever part),
    batched over robots.  Returns (pos_des', xref (B,N,12), contact (B,4,N) uint8,
    r_feet (B,N,4,3))."""
    x0 = np.asarray(x0, np.float64)
    B = x0.shape[0]
    pos_des = np.array(pos_des, np.float64, copy=True)
    cmd = np.asarray(cmd, np.float64)
    t_now = np.asarray(t_now, np.float64)
    period, duty, offs = gait[:, 0], gait[:, 1], gait[:, 2:6]
    vx, vy, z_des, wz = cmd[:, 0], cmd[:, 1], cmd[:, 2], cmd[:, 3]
    px, py, yaw = x0[:, 0], x0[:, 1], x0[:, 5]

    # :47-60 clamp the desired position to within 0.1 m of the current COM (x, y); z commanded
    for a, cur in ((0, px), (1, py)):
        hi = pos_des[:, a] - cur > MAX_POS_ERROR
        pos_des[hi, a] = cur[hi] + MAX_POS_ERROR
        lo = cur - pos_des[:, a] > MAX_POS_ERROR
        pos_des[lo, a] = cur[lo] - MAX_POS_ERROR
    pos_des[:, 2] = z_des

    # :66-104 x_ref over t = dt .. N dt
    t_vec = (np.arange(N) + 1) * dt
    Rz0 = rz(yaw)
    v_world = np.einsum('bij,bj->bi', Rz0, np.stack([vx, vy, np.zeros(B)], -1))   # :73
    pos_traj = pos_des[:, :, None] + v_world[:, :, None] * t_vec[None, None, :]   # (B,3,N) :86
    yaw_traj = yaw[:, None] + wz[:, None] * t_vec[None, :]                        # :98
    xref = np.zeros((B, N, 12))
    xref[:, :, 0:3] = pos_traj.transpose(0, 2, 1)
    xref[:, :, 5] = yaw_traj
    xref[:, :, 6:9] = v_world[:, None, :]
    xref[:, :, 11] = wz[:, None]

    # :106 contact table at mid-step times (gait.py:29-30)
    t_mid = t_now[:, None] + np.arange(N)[None, :] * dt
    t_mid = t_mid + dt / 2
    contact = phase_mask(t_mid, period, duty, offs).astype(np.uint8)

    # :108-201 foot levers.  Mask at the start of each step (compute_current_mask(time_now +
    # i dt) = compute_contact_table(t, 0, 1), gait.py:21-24); at take-off the next touchdown
    # is predicted from the dummy model's pose at that step (gait.py:40-74).
    t_start = t_now[:, None] + np.arange(N)[None, :] * dt
    mask = phase_mask(t_start, period, duty, offs)                                  # (B,4,N)
    R_wb = np.swapaxes(rot_zyx(x0[:, 3:6]), -1, -2)          # go2.R_world_to_body (:125)
    v_body = np.einsum('bij,bj->bi', R_wb, v_world)          # :126-130 (dq[0:3])
    t_swing = (1.0 - duty) * period                          # gait.py:18-19
    t_stance = duty * period
    pred_time = (t_swing + 0.5 * t_stance) / 2.0             # gait.py:54-55
    r_feet = np.zeros((B, N, 4, 3))
    r_next = np.array(foot_lever, np.float64, copy=True)     # :113
    prev = np.full((B, 4), 2)                                # :115
    for i in range(N):
        cur = mask[:, :, i].astype(int)
        base = pos_traj[:, :, i]                             # dummy base_pos (:134)
        Rzi = rz(yaw_traj[:, i])                             # dummy R_z (update_model_simplified)
        takeoff = (cur != prev) & (cur == 0)
        touchdown = (cur != prev) & (cur == 1)
        same = cur == prev
        for leg in range(4):
            # gait.py:41-72 touchdown prediction
            hip_w = np.einsum('bij,j->bi', Rzi, hip[leg])
            nominal = np.stack([base[:, 0] + hip_w[:, 0], base[:, 1] + hip_w[:, 1],
                                np.full(B, TD_HEIGHT)], -1)
            drift = np.stack([v_body[:, 0] * pred_time, v_body[:, 1] * pred_time, np.zeros(B)], -1)
            dtheta = wz * pred_time
            r_xy = nominal[:, 0:2] - base[:, 0:2]
            rot = np.stack([-dtheta * r_xy[:, 1], dtheta * r_xy[:, 0], np.zeros(B)], -1)
            td = nominal + drift + rot
            to = takeoff[:, leg]
            r_next[to, leg] = td[to] - base[to]              # :139-140
            r_feet[to, i, leg] = 0.0                         # :142
            tdn = touchdown[:, leg]
            r_feet[tdn, i, leg] = r_next[tdn, leg]           # :146
            sm = same[:, leg]
            r_feet[sm, i, leg] = r_feet[sm, i - 1, leg]      # :150 (i >= 1 here: prev starts at 2)
        prev = cur
    return pos_des, xref, contact, r_feet
