"""GPU: the whole tick in closed loop on the device (generate_traj -> build_dynamics -> warm
solve -> cmpc_srb_step), B robots trotting under commanded velocities -- the loop shape of
test_MPC.py:160-236 with the single-rigid-body stand-in for MuJoCo (absent from the image).

Properties checked (there is no reference trajectory to compare with: the reference's plant is
MuJoCo): every solve KKT-verified, the robots stay up (COM height, roll/pitch bounded), they
track the commanded body velocity, and a HIP-graph replay of the tick is bit-identical to the
eager tick."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _command(B, rng):
    return np.stack([rng.uniform(-0.5, 0.5, B), rng.uniform(-0.2, 0.2, B),
                     np.full(B, 0.27), rng.uniform(-1.0, 1.0, B)], 1)


def test_closed_loop_trot_tracks_command(plan):
    import torch
    from cmpc.closed_loop import ClosedLoop
    B = 512
    rng = np.random.default_rng(0)
    cl = ClosedLoop(B, plan=plan, seed=1)
    cmd = _command(B, rng)
    cl.set_command(cmd)
    vb_log, bad = [], 0
    for k in range(96):                      # 2 s of simulated time (MPC_DT = 1/48 s)
        cl.tick()
        torch.cuda.synchronize()
        bad += int((cl.status != 1).sum())
        if k >= 72:
            x = cl.x.cpu().numpy().astype(np.float64)
            c, s = np.cos(x[:, 5]), np.sin(x[:, 5])
            vb_log.append(np.stack([c * x[:, 6] + s * x[:, 7], -s * x[:, 6] + c * x[:, 7]], 1))
    x = cl.x.cpu().numpy()
    assert bad == 0, bad
    assert np.all(np.isfinite(x))
    assert np.all(np.abs(x[:, 2] - 0.27) < 0.05), (x[:, 2].min(), x[:, 2].max())
    assert np.all(np.abs(x[:, 3:5]) < 0.3), np.abs(x[:, 3:5]).max()
    vb = np.mean(vb_log, 0)                  # mean body velocity over the last 0.5 s
    err = np.abs(vb - cmd[:, :2])
    assert err.mean() < 0.05 and err.max() < 0.25, (err.mean(), err.max())


def test_graph_replay_matches_eager(plan):
    import torch
    from cmpc.closed_loop import ClosedLoop
    B = 256
    rng = np.random.default_rng(2)
    cmd = _command(B, rng)
    a, b = ClosedLoop(B, plan=plan, seed=3), ClosedLoop(B, plan=plan, seed=3)
    a.set_command(cmd); b.set_command(cmd)
    for _ in range(3):
        a.tick(); b.tick()
    b.capture()
    for _ in range(5):
        a.tick(); b.tick()
    torch.cuda.synchronize()
    assert torch.equal(a.x, b.x) and torch.equal(a.w, b.w) and torch.equal(a.t, b.t)


# test_MPC.py:37-47 CMD_SCHEDULE: (t_start, t_end, x_vel, y_vel, z_pos, yaw_rate)
CMD_SCHEDULE = [(0.0, 1.0, 0.7, 0.0, 0.27, 0.0), (1.0, 1.5, 0.0, 0.0, 0.27, 0.0),
                (1.5, 3.0, 0.0, 0.3, 0.27, 0.0), (3.0, 4.0, 0.0, 0.0, 0.27, 0.0),
                (4.0, 6.0, 0.0, 0.0, 0.27, 2.0), (6.0, 6.5, 0.0, 0.0, 0.27, 0.0),
                (6.5, 8.0, 0.6, 0.0, 0.27, 2.0), (8.0, 9.0, 0.8, 0.0, 0.27, 0.0),
                (9.0, 10.0, 0.0, 0.0, 0.27, 0.0)]


def _body_cmd(t):
    """test_MPC.py:82-92 get_body_cmd."""
    for (t0, t1, vx, vy, z, wz) in CMD_SCHEDULE:
        if t0 <= t < t1:
            return vx, vy, z, wz
    return 0.0, 0.0, 0.27, 0.0


def test_reference_command_schedule(plan):
    """The reference demo's 10 s command schedule (test_MPC.py:37-47, trot 3 Hz / 0.6), for 128
    robots with random headings in closed loop: every phase's command is tracked at its end."""
    import torch
    from cmpc.closed_loop import ClosedLoop
    B = 128
    cl = ClosedLoop(B, plan=plan, seed=4)
    n_ticks = int(round(10.0 / cl.dt))
    log = []
    for k in range(n_ticks):
        t = k * cl.dt
        cl.set_command(np.tile(_body_cmd(t), (B, 1)))
        cl.tick()
        torch.cuda.synchronize()
        assert int((cl.status != 1).sum()) == 0, k
        x = cl.x.cpu().numpy().astype(np.float64)
        c, s = np.cos(x[:, 5]), np.sin(x[:, 5])
        log.append((t + cl.dt, c * x[:, 6] + s * x[:, 7], -s * x[:, 6] + c * x[:, 7], x[:, 11],
                    x[:, 2], np.abs(x[:, 3:5]).max(1)))
    for (t0, t1, vx, vy, z, wz) in CMD_SCHEDULE:
        tail = [e for e in log if t1 - 0.25 <= e[0] < t1]      # the phase's last quarter second
        mvx = np.mean([e[1] for e in tail], 0)
        mvy = np.mean([e[2] for e in tail], 0)
        mwz = np.mean([e[3] for e in tail], 0)
        assert np.abs(mvx - vx).max() < 0.15, (t0, np.abs(mvx - vx).max())
        # turning while walking: the reference velocity is frozen in the world frame over the
        # horizon (com_trajectory.py:72-92), so a lateral lag ~ vx wz is inherent to the MPC
        assert np.abs(mvy - vy).max() < 0.15 + 0.05 * abs(vx * wz), (t0, np.abs(mvy - vy).max())
        assert np.abs(mwz - wz).max() < 0.3, (t0, np.abs(mwz - wz).max())
    assert min(e[4].min() for e in log) > 0.22 and max(e[4].max() for e in log) < 0.32
    assert max(e[5].max() for e in log) < 0.3
