"""CPU: oracle/traj_ref.py (batched restatement of ComTraj.generate_traj, com_trajectory.py:27-207,
and gait.py:21-74) against the reference's own outputs (tests/golden/traj_ticks.npz, produced by
running the reference's generate_traj; see tests/golden/make_golden.py)."""
import numpy as np

from oracle import traj_ref
from parity_util import load_fixture


def _tick(d, i):
    N = int(d["N"][i])
    out = traj_ref.generate_traj(d["x0"][i:i + 1], d["pos_des_in"][i:i + 1], d["cmd"][i:i + 1],
                                 d["t_now"][i:i + 1], d["gait"][i:i + 1], d["foot_lever"][i:i + 1],
                                 d["hip"], float(d["dt"][i]), N)
    return N, [o[0] for o in out]


def test_oracle_matches_reference_generate_traj():
    d = load_fixture("traj_ticks.npz")
    assert len(d["N"]) >= 48 and set(d["N"].tolist()) == {8, 16}
    for i in range(len(d["N"])):
        N, (pd, xref, ct, rf) = _tick(d, i)
        np.testing.assert_array_equal(ct, d["contact"][i][:, :N])          # bit-exact schedule
        np.testing.assert_allclose(pd, d["pos_des_out"][i], rtol=0, atol=1e-15)
        np.testing.assert_allclose(xref, d["xref"][i][:N], rtol=0, atol=1e-14)
        np.testing.assert_allclose(rf, d["r_feet"][i][:N], rtol=0, atol=1e-14)


def test_fixture_covers_lever_cases():
    """The fixture exercises every branch of the lever recursion (com_trajectory.py:136-198):
    initial lever kept through a stance run, take-off (0), touchdown with a predicted lever, and
    the mid-step/start-of-step mask mismatch (stance in the QP with a zero lever)."""
    d = load_fixture("traj_ticks.npz")
    init_kept = pred = mismatch = 0
    for i in range(len(d["N"])):
        N = int(d["N"][i])
        rf, fl, ct = d["r_feet"][i][:N], d["foot_lever"][i], d["contact"][i][:, :N]
        for leg in range(4):
            nz = np.abs(rf[:, leg]).sum(-1) > 0
            init_kept += int(np.sum(np.all(rf[:, leg] == fl[leg], axis=-1)))
            pred += int(np.sum(nz & ~np.all(rf[:, leg] == fl[leg], axis=-1)))
            mismatch += int(np.sum((ct[leg] == 1) & ~nz))
    assert init_kept > 0 and pred > 0 and mismatch > 0, (init_kept, pred, mismatch)


def test_pos_des_state_carries_across_ticks():
    """ComTraj.pos_des_world persists between ticks (com_trajectory.py:13, :47-60): each tick's
    input state is the previous tick's output for the same robot."""
    d = load_fixture("traj_ticks.npz")
    x0 = d["x0"]
    carried = 0
    for i in range(1, len(d["N"])):
        same_robot = np.array_equal(d["gait"][i], d["gait"][i - 1]) and d["t_now"][i] > d["t_now"][i - 1]
        if same_robot:
            np.testing.assert_array_equal(d["pos_des_in"][i], d["pos_des_out"][i - 1])
            carried += 1
    assert carried >= 40
    # the clamp keeps x/y within 0.1 m of the COM
    assert np.all(np.abs(d["pos_des_out"][:, :2] - x0[:, :2]) <= 0.1 + 1e-12)
