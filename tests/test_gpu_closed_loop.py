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
