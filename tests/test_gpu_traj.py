"""GPU: on-device reference trajectory / contact table / foot levers (cmpc_generate_traj,
SURVEY.md 8(f) row 2) against the reference's own generate_traj outputs
(tests/golden/traj_ticks.npz) and the batched oracle (oracle/traj_ref.py), and the whole
on-device tick (generate_traj -> build_dynamics -> solve) against the oracle chain + the
KKT-certified float64 solver.

Tolerances: the contact table and the desired-position state are computed in float64 with the
reference's operation order and must match exactly.  x_ref and the levers are float64 rounded
once to fp32: an entry may differ from the float64 reference by one fp32 rounding (2^-23
relative) plus 1e-12 absolute.  The solve keeps the QP parity bar, |dU|inf/|U*|inf <= 1e-4."""
import numpy as np
import pytest

from parity_util import load_fixture

pytestmark = pytest.mark.gpu

REL = 2.0 ** -23


def _close(gpu, ref):
    ref = np.asarray(ref, np.float64)
    err = np.abs(np.asarray(gpu, np.float64) - ref)
    bad = err > REL * np.abs(ref) + 1e-12
    if np.any(bad):
        print("max err", err.max(), "at", np.argwhere(bad)[:5])
    return not np.any(bad)


def _dev(a, torch, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype or torch.float32).cuda()


def _run(plan, torch, x0, pos_des, cmd, t_now, gait, lever, hip, dt):
    pd = _dev(pos_des, torch, torch.float64)
    xref, ct, rf = plan.generate_traj(_dev(x0, torch), pd, _dev(cmd, torch),
                                      _dev(t_now, torch, torch.float64),
                                      _dev(gait, torch, torch.float64), _dev(lever, torch),
                                      _dev(hip, torch), dt)
    torch.cuda.synchronize()
    return pd.cpu().numpy(), xref.cpu().numpy(), ct.cpu().numpy(), rf.cpu().numpy()


@pytest.mark.parametrize("N", [16, 8])
def test_golden_reference_generate_traj(plan, N):
    """Every fixture tick of horizon N in one batch (robots with different gaits and times)."""
    import torch
    from cmpc import Plan, SolverParams
    d = load_fixture("traj_ticks.npz")
    sel = np.nonzero(d["N"] == N)[0]
    assert len(sel) > 0
    dts = np.unique(d["dt"][sel])
    pl = plan if N == plan.params.N else Plan(SolverParams(N=N, max_batch=1024))
    for dt in dts:                       # dt is one scalar per call
        s = sel[d["dt"][sel] == dt]
        pd, xref, ct, rf = _run(pl, torch, d["x0"][s], d["pos_des_in"][s], d["cmd"][s],
                                d["t_now"][s], d["gait"][s], d["foot_lever"][s], d["hip"], float(dt))
        np.testing.assert_array_equal(ct, d["contact"][s][:, :, :N])
        np.testing.assert_array_equal(pd, d["pos_des_out"][s])
        assert _close(xref, d["xref"][s][:, :N])
        assert _close(rf, d["r_feet"][s][:, :N])


@pytest.mark.parametrize("mixed", [False, True])
def test_batched_vs_oracle(plan, mixed):
    import torch
    from cmpc import synth
    from oracle import traj_ref
    B = 4096
    t = synth.make_tick_inputs(B, seed=21 + mixed, mixed=mixed)
    # exact phase ties: a block of robots at step-aligned times with duty 1/2 (phase == duty)
    t["t_now"][:256] = np.arange(256) * t["dt"]
    t["gait"][:256, 1] = 0.5
    t["t_now"][256:512] = 1000.0 + np.arange(256) * t["dt"] * 0.5   # large times
    args = [t[k] for k in ("x0", "pos_des", "cmd", "t_now", "gait", "foot_lever")]
    pd, xref, ct, rf = _run(plan, torch, *args, t["hip"], t["dt"])
    pd_o, xref_o, ct_o, rf_o = traj_ref.generate_traj(*args, t["hip"], t["dt"], 16)
    np.testing.assert_array_equal(ct, ct_o)
    np.testing.assert_array_equal(pd, pd_o)
    assert _close(xref, xref_o)
    assert _close(rf, rf_o)


def test_pos_des_state_in_place_over_ticks(plan):
    """Three ticks with the desired-position state kept on the device (ComTraj.pos_des_world,
    com_trajectory.py:13, :47-60) match three oracle ticks."""
    import torch
    from cmpc import synth
    from oracle import traj_ref
    t = synth.make_tick_inputs(512, seed=5, mixed=True)
    pd = _dev(t["pos_des"], torch, torch.float64)
    pd_o = t["pos_des"].copy()
    x0, tn = t["x0"].copy(), t["t_now"].copy()
    rng = np.random.default_rng(0)
    hip = _dev(t["hip"], torch)
    for _ in range(3):
        xr, ct, rf = plan.generate_traj(_dev(x0, torch), pd, _dev(t["cmd"], torch),
                                        _dev(tn, torch, torch.float64),
                                        _dev(t["gait"], torch, torch.float64),
                                        _dev(t["foot_lever"], torch), hip, t["dt"])
        pd_o, xr_o, ct_o, rf_o = traj_ref.generate_traj(x0, pd_o, t["cmd"], tn, t["gait"],
                                                        t["foot_lever"], t["hip"], t["dt"], 16)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(pd.cpu().numpy(), pd_o)
        np.testing.assert_array_equal(ct.cpu().numpy(), ct_o)
        assert _close(xr.cpu().numpy(), xr_o)
        x0 = np.float32(x0 + rng.normal(0, 0.08, x0.shape)).astype(np.float64)
        tn = tn + t["dt"]


def test_full_tick_on_device_vs_oracle_chain(plan):
    """generate_traj -> build_dynamics -> solve, all on the device, against the oracle chain
    (traj_ref -> closed-form discretisation -> KKT-certified float64 solve)."""
    import torch
    from cmpc import synth
    from oracle import mpc_qp, tight_solver, traj_ref
    B = 24
    t = synth.make_tick_inputs(B, seed=9, mixed=True)
    args = [t[k] for k in ("x0", "pos_des", "cmd", "t_now", "gait", "foot_lever")]
    x0d = _dev(t["x0"], torch)
    pd = _dev(t["pos_des"], torch, torch.float64)
    xref, ct, rf = plan.generate_traj(x0d, pd, _dev(t["cmd"], torch),
                                      _dev(t["t_now"], torch, torch.float64),
                                      _dev(t["gait"], torch, torch.float64),
                                      _dev(t["foot_lever"], torch), _dev(t["hip"], torch), t["dt"])
    Ad, Bd, gd = plan.build_dynamics(_dev(t["m"], torch), _dev(t["I_world"], torch), rf, xref,
                                     t["dt"])
    w, st, it = plan.solve(Ad, Bd, gd, x0d, xref, ct)
    torch.cuda.synchronize()
    w, st = w.cpu().numpy(), st.cpu().numpy()
    assert np.all(st == 1), st
    _, xr_o, ct_o, rf_o = traj_ref.generate_traj(*args, t["hip"], t["dt"], 16)
    np.testing.assert_array_equal(ct.cpu().numpy(), ct_o)
    Ad_o, Bd_o, gd_o = synth.discretize(t["m"], t["I_world"], rf_o, xr_o[:, :, 5].mean(1), t["dt"])
    worst = 0.0
    for i in range(B):
        qp = mpc_qp.build_qp(Ad_o[i], Bd_o[i], gd_o[i], t["x0"][i], xr_o[i].T, ct_o[i])
        Ur = tight_solver.solve(qp)["w"][192:]
        U = w[i, 192:].astype(np.float64)
        worst = max(worst, float(np.max(np.abs(U - Ur)) / np.max(np.abs(Ur))))
    assert worst <= 1e-4, worst
