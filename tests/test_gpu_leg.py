"""GPU: the leg controller on the device (cmpc_leg_torque) against the
reference's own LegController over consecutive 1 kHz ticks (tests/golden/leg_ticks.npz) and the
batched oracle (oracle/leg_ref.py), with the controller memory kept on the device.

Tolerance: both sides are float64; the device factors M by Cholesky where the reference inverts
it by LU, so torques agree to |d tau| <= 1e-9 (1 + |tau|)."""
import numpy as np
import pytest

from parity_util import load_fixture
from test_leg import leg_inputs, tick_index

pytestmark = pytest.mark.gpu

TOL = 1e-9


def _dev(x, torch, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype or torch.float64).cuda()


def _call(plan, torch, inp, state, tau_max):
    import torch as T
    args = {k: _dev(v, torch) for k, v in inp.items() if k != "force"}
    force = _dev(inp["force"], torch, T.float32)
    return plan.leg_torque(args["t"], args["gait"], force, args["J_foot"], args["J_full"],
                           args["M"], args["C"], args["g"], args["dq"], args["Jdot_dq"],
                           args["foot_pos"], args["foot_vel"], args["body"], args["hip"], state,
                           tau_max=tau_max)


def test_golden_reference_leg_controller(plan):
    import torch
    from cmpc import leg_state
    d = load_fixture("leg_ticks.npz")
    ti = tick_index(d)
    state = leg_state(ti.shape[1])
    worst = 0.0
    for k in range(ti.shape[0]):
        tau = _call(plan, torch, leg_inputs(d, ti[k]), state, 0.0).cpu().numpy()
        ref = d["tau"][ti[k]]
        worst = max(worst, float(np.max(np.abs(tau - ref) / (1 + np.abs(ref)))))
    assert worst <= TOL, worst


def test_batched_vs_oracle_with_clip(plan):
    """4,096 robots (random SPD M, random gaits and times) over 60 ticks, clip at 45 N m."""
    import torch
    from cmpc import leg_state
    from oracle import leg_ref
    rng = np.random.default_rng(3)
    B = 4096
    A = rng.normal(0, 1, (B, 18, 18))
    base = dict(J_foot=rng.normal(0, 0.2, (B, 4, 3, 3)), J_full=rng.normal(0, 0.2, (B, 4, 3, 18)),
                M=A @ np.swapaxes(A, 1, 2) / 18 + np.eye(18) * 0.3, C=rng.normal(0, 0.1, (B, 18, 18)),
                hip=np.array([[0.19, 0.14, 0], [0.19, -0.14, 0], [-0.19, 0.14, 0], [-0.19, -0.14, 0.0]]))
    gait = np.concatenate([1.0 / rng.uniform(2, 5, (B, 1)), rng.uniform(0.4, 0.8, (B, 1)),
                           rng.uniform(0, 1, (B, 4))], 1)
    t = rng.uniform(0, 5, B)
    state_d = leg_state(B)
    state_o = np.zeros((B, 4, 8)); state_o[:, :, 0] = 2
    worst = 0.0
    for _ in range(60):
        inp = dict(t=t, gait=gait, force=np.float32(rng.normal(0, 60, (B, 12))).astype(np.float64),
                   g=rng.normal(0, 3, (B, 18)), dq=rng.normal(0, 1, (B, 18)),
                   Jdot_dq=rng.normal(0, 0.3, (B, 4, 3)), foot_pos=rng.normal(0, 0.3, (B, 4, 3)),
                   foot_vel=rng.normal(0, 0.3, (B, 4, 3)),
                   body=np.concatenate([rng.normal(0, 0.5, (B, 9)), rng.uniform(-3, 3, (B, 2)),
                                        rng.normal(0, 0.5, (B, 4)), np.zeros((B, 1))], 1), **base)
        tau = _call(plan, torch, inp, state_d, 45.0).cpu().numpy()
        tau_o, state_o = leg_ref.leg_torque(**inp, state=state_o, tau_max=45.0)
        worst = max(worst, float(np.max(np.abs(tau - tau_o) / (1 + np.abs(tau_o)))))
        t = t + 0.004
    assert np.abs(tau).max() <= 45.0
    assert worst <= TOL, worst
    np.testing.assert_allclose(state_d.cpu().numpy(), state_o, rtol=0, atol=1e-12)


def test_stance_forces_from_solver_output(plan):
    """Stance legs take U[:, 0] straight from the solver's w (row stride 24 N, offset 12 N)."""
    import torch
    from cmpc import leg_state, solve_batch, synth
    b = synth.make_config(1, B=64)
    w, st, _ = solve_batch(b, plan=plan)
    wd = torch.as_tensor(w).cuda()
    B = 64
    rng = np.random.default_rng(5)
    J = rng.normal(0, 0.2, (B, 4, 3, 3))
    gait = np.tile([1 / 3.0, 1.0, 0, 0, 0, 0], (B, 1))          # duty 1: every leg in stance
    z = lambda *s: torch.zeros(s, dtype=torch.float64, device="cuda")  # noqa: E731
    Jd = _dev(J, torch)
    M = torch.eye(18, dtype=torch.float64, device="cuda").repeat(B, 1, 1)
    tau = plan.leg_torque(_dev(np.zeros(B), torch), _dev(gait, torch), wd[:, 192:], Jd,
                          z(B, 4, 3, 18), M, z(B, 18, 18), z(B, 18), z(B, 18), z(B, 4, 3),
                          z(B, 4, 3), z(B, 4, 3), z(B, 16), z(4, 3), leg_state(B), tau_max=0.0)
    U0 = w[:, 192:204].astype(np.float64).reshape(B, 4, 3)
    ref = np.einsum('blji,blj->bli', J, -U0).reshape(B, 12)     # J' (-f), leg_controller.py:101
    np.testing.assert_allclose(tau.cpu().numpy(), ref, rtol=1e-12, atol=1e-12)
