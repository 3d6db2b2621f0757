"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- batched restatement of the reference's leg controller
tick: the consumer of the QP's first forces ("stance torque mapping").

Restates, in float64 NumPy, ``LegController.compute_leg_torque`` (``convex_mpc/leg_controller.py:
43-112``) for the four legs of a batch of robots, with the swing planning it calls at take-off
(``Gait.compute_swing_traj_and_touchdown`` + ``make_swing_trajectory``, ``gait.py:77-174``) and the
motor saturation of the loop (``np.clip(tau, -TAU_MAX, TAU_MAX)``, ``test_MPC.py:227-228``).  The
Pinocchio quantities the reference reads are inputs (``go2_robot_data.py:271-360``).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this file; the
product path never does.  Pinned against ``tests/golden/leg_ticks.npz``, produced by running the
reference's own ``LegController`` and ``Gait`` (tests/golden/make_golden.py).

Batched layouts (the C-ABI's, include/cmpc.h ``cmpc_leg_torque``):
  t (B,) f64; gait (B,6) = [period, duty, offsets FL FR RL RR]; force (B,12) = U[:, 0];
  J_foot (B,4,3,3); J_full (B,4,3,18); M, C (B,18,18); g, dq (B,18); Jdot_dq, foot_pos,
  foot_vel (B,4,3); body (B,16) = [base_pos(3), pos_com(3), vel_com(3), yaw, yaw_rate_des,
  x_pos_des, y_pos_des, x_vel_des, y_vel_des, 0]; hip (4,3);
  state (B,4,8) in/out = [last_mask, takeoff_time, p0(3), pf(3)]  (last_mask 2 = never run)
  -> tau (B,12).
"""
from __future__ import annotations

import numpy as np

KP_SWING = 500.0         # leg_controller.py:10
KD_SWING = 200.0         # leg_controller.py:11
HEIGHT_SWING = 0.1       # gait.py:9
TD_HEIGHT = 0.02         # gait.py:116
TAU_MAX = 45.0           # test_MPC.py (TAU_MAX), applied at :227-228


def stance_now(t, period, duty, offsets):
    """gait.py:21-37 compute_current_mask(t) = compute_contact_table(t, 0, 1)[:, 0]."""
    ph = np.mod(offsets + (t + 0.0 / 2)[:, None] / period[:, None], 1.0)
    return (ph < duty[:, None]).astype(int)


def touchdown(body, hip, foot_leg, period, duty, leg):
    """gait.py:77-133 compute_swing_traj_and_touchdown: the predicted touchdown (B,3)."""
    B = body.shape[0]
    base = body[:, 0:3]
    com, vcom = body[:, 3:6], body[:, 6:9]
    yaw, yaw_rate = body[:, 9], body[:, 10]
    xpd, ypd, xvd, yvd = body[:, 11], body[:, 12], body[:, 13], body[:, 14]
    c, s = np.cos(yaw), np.sin(yaw)
    h = hip[leg]
    hip_w = np.stack([base[:, 0] + (c * h[0] - s * h[1] + 0.0 * h[2]),
                      base[:, 1] + (s * h[0] + c * h[1] + 0.0 * h[2])], -1)
    t_swing = (1 - duty) * period
    t_stance = duty * period
    T = t_swing + 0.5 * t_stance
    pred = T / 2.0
    k_v_x, k_p_x = 0.4 * T, 0.1
    k_v_y, k_p_y = 0.2 * T, 0.05
    nominal = np.stack([hip_w[:, 0], hip_w[:, 1], np.full(B, TD_HEIGHT)], -1)
    drift = np.stack([xvd * pred, yvd * pred, np.zeros(B)], -1)
    pcorr = np.stack([k_p_x * (com[:, 0] - xpd), k_p_y * (com[:, 1] - ypd), np.zeros(B)], -1)
    vcorr = np.stack([k_v_x * (vcom[:, 0] - xvd), k_v_y * (vcom[:, 1] - yvd), np.zeros(B)], -1)
    dth = yaw_rate * pred
    r_xy = nominal[:, 0:2] - base[:, 0:2]
    rot = np.stack([-dth * r_xy[:, 1], dth * r_xy[:, 0], np.zeros(B)], -1)
    return nominal + drift + pcorr + vcorr + rot


def swing_eval(p0, pf, T, t):
    """gait.py:138-172 make_swing_trajectory(...)(t): (p, v, a), each (B,3)."""
    s = np.clip(t / T, 0.0, 1.0)[:, None]
    dp = pf - p0
    mj = 10 * s**3 - 15 * s**4 + 6 * s**5
    dmj = 30 * s**2 - 60 * s**3 + 30 * s**4
    d2mj = 60 * s - 180 * s**2 + 120 * s**3
    Tc = T[:, None]
    p = p0 + dp * mj
    v = (dp * dmj) / Tc
    a = (dp * d2mj) / (Tc**2)
    s1 = s[:, 0]
    b = 64 * s1**3 * (1 - s1)**3
    db = 192 * s1**2 * (1 - s1)**2 * (1 - 2 * s1)
    d2b = 192 * (2 * s1 * (1 - s1)**2 * (1 - 2 * s1) - 2 * s1**2 * (1 - s1) * (1 - 2 * s1)
                 - 2 * s1**2 * (1 - s1)**2)
    p[:, 2] += HEIGHT_SWING * b
    v[:, 2] += HEIGHT_SWING * db / T
    a[:, 2] += HEIGHT_SWING * d2b / (T**2)
    return p, v, a


def leg_torque(t, gait, force, J_foot, J_full, M, C, g, dq, Jdot_dq, foot_pos, foot_vel, body,
               hip, state, tau_max=TAU_MAX):
    """leg_controller.py:43-112 for legs FL FR RL RR (test_MPC.py:199-225) + the clip of
    test_MPC.py:227-228.  Returns (tau (B,12), state')."""
    t = np.asarray(t, np.float64)
    B = t.shape[0]
    state = np.array(state, np.float64, copy=True)
    period, duty, offs = gait[:, 0], gait[:, 1], gait[:, 2:6]
    mask = stance_now(t, period, duty, offs)                 # :59
    h = np.einsum('bij,bj->bi', C, dq) + g                   # (C @ dq + g), :98
    Minv = np.linalg.inv(M)                                  # :87
    t_swing = (1 - duty) * period
    tau = np.zeros((B, 12))
    for leg in range(4):
        cur = mask[:, leg]
        last = state[:, leg, 0]
        to = (last != cur) & (cur == 0)                       # :67
        if np.any(to):
            pf = touchdown(body, hip, foot_pos[:, leg], period, duty, leg)
            state[to, leg, 1] = t[to]
            state[to, leg, 2:5] = foot_pos[to, leg]           # p0 = foot position at take-off
            state[to, leg, 5:8] = pf[to]
        sw = cur == 0
        # swing (:75-98)
        p, v, a = swing_eval(state[:, leg, 2:5], state[:, leg, 5:8], t_swing, t - state[:, leg, 1])
        pos_err = p - foot_pos[:, leg]
        vel_err = v - foot_vel[:, leg]
        Jf = J_full[:, leg]
        Lam = np.linalg.inv(np.einsum('bij,bjk,blk->bil', Jf, Minv, Jf))
        f_ff = np.einsum('bij,bj->bi', Lam, a - Jdot_dq[:, leg])
        fsw = KP_SWING * pos_err + KD_SWING * vel_err + f_ff
        tau_sw = np.einsum('bji,bj->bi', J_foot[:, leg], fsw) + h[:, 6 + 3 * leg:9 + 3 * leg]
        # stance (:100-101): J' (-f)
        tau_st = np.einsum('bji,bj->bi', J_foot[:, leg], -force[:, 3 * leg:3 * leg + 3])
        tau[:, 3 * leg:3 * leg + 3] = np.where(sw[:, None], tau_sw, tau_st)
        state[:, leg, 0] = cur                                # :104
    if tau_max > 0:
        tau = np.clip(tau, -tau_max, tau_max)
    return tau, state
