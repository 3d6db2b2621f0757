"""CPU: oracle/leg_ref.py (batched restatement of LegController.compute_leg_torque,
leg_controller.py:43-112, with the swing planning of gait.py:77-174) against the reference's own
outputs over consecutive 1 kHz ticks (tests/golden/leg_ticks.npz, made by running the reference's
LegController; see tests/golden/make_golden.py)."""
import numpy as np

from oracle import leg_ref
from parity_util import load_fixture


def leg_inputs(d, idx):
    """Batched kernel/oracle inputs of fixture ticks `idx` (one tick per robot)."""
    r = d["robot"][idx]
    f = lambda k: d[k][idx].astype(np.float64)  # noqa: E731
    return dict(t=d["t"][idx], gait=d["gait"][idx], force=f("force"),
                J_foot=d["J_foot"][r].astype(np.float64), J_full=d["J_full"][r].astype(np.float64),
                M=d["M"][r].astype(np.float64), C=d["C"][r].astype(np.float64), g=f("g"),
                dq=f("dq"), Jdot_dq=f("Jdot_dq"), foot_pos=f("foot_pos"),
                foot_vel=f("foot_vel"), body=f("body"), hip=d["hip"].astype(np.float64))


def tick_index(d):
    """(n_ticks, n_robots) fixture row of tick k of robot r."""
    robots = np.unique(d["robot"])
    return np.stack([np.nonzero(d["robot"] == r)[0] for r in robots], 1)


def test_oracle_matches_reference_leg_controller():
    d = load_fixture("leg_ticks.npz")
    ti = tick_index(d)
    state = np.zeros((ti.shape[1], 4, 8)); state[:, :, 0] = 2
    worst = 0.0
    for k in range(ti.shape[0]):
        tau, state = leg_ref.leg_torque(**leg_inputs(d, ti[k]), state=state, tau_max=0.0)
        ref = d["tau"][ti[k]]
        worst = max(worst, float(np.max(np.abs(tau - ref) / (1 + np.abs(ref)))))
    assert worst < 1e-10, worst


def test_fixture_covers_swing_and_stance():
    d = load_fixture("leg_ticks.npz")
    ti = tick_index(d)
    state = np.zeros((ti.shape[1], 4, 8)); state[:, :, 0] = 2
    swing = stance = takeoffs = 0
    for k in range(ti.shape[0]):
        prev = state[:, :, 0].copy()
        _, state = leg_ref.leg_torque(**leg_inputs(d, ti[k]), state=state, tau_max=0.0)
        swing += int((state[:, :, 0] == 0).sum()); stance += int((state[:, :, 0] == 1).sum())
        takeoffs += int(((prev == 1) & (state[:, :, 0] == 0)).sum())
    assert swing > 300 and stance > 300 and takeoffs >= 5, (swing, stance, takeoffs)
