"""GPU: small-batch team mode (cmpc_team.hip, cmpc_plan_set_team) -- four waves per QP split
the condensation, the inversion and the matrix-vector products.  Same algorithm, same parity
bar as the one-wave kernels: max |U_gpu - U*| / max |U*| <= 1e-4 per instance against the
KKT-certified optimum (oracle/tight_solver.py), every instance status 1.

Each test forces the mode (set_team(2**40) = always team, set_team(0) = never), so the team
kernels are exercised at batch sizes the automatic rule would give to the one-wave kernels too.
"""
import numpy as np
import pytest
import torch

from parity_util import (load_fixture, fixture_batch, rel_err_U, split_w, rollout64,
                         feasibility)

pytestmark = pytest.mark.gpu
TOL_U = 1e-4
ALWAYS = 1 << 40


@pytest.fixture(scope="module")
def team_plan():
    from cmpc import Plan, SolverParams
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    p = Plan(SolverParams(max_batch=65536))
    p.set_team(ALWAYS)
    return p


@pytest.fixture(scope="module")
def wave_plan():
    from cmpc import Plan, SolverParams
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    p = Plan(SolverParams(max_batch=65536))
    p.set_team(0)
    return p


@pytest.mark.parametrize("name", ["qp_cfg1.npz", "qp_cfg2.npz", "qp_nc192.npz", "qp_hard.npz"])
def test_team_fixture_parity(team_plan, name):
    from cmpc import solve_batch
    fx = load_fixture(name)
    batch = fixture_batch(fx)
    w, st, it = solve_batch(batch, plan=team_plan)
    assert np.all(st == 1), (st, it)
    err = rel_err_U(w, fx["w"])
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()))
    Xg, Ug = split_w(w.astype(np.float64))
    assert np.max(np.abs(Xg - rollout64(batch, Ug))) < 1e-4
    assert feasibility(batch, Ug).max() < 1e-3


def test_team_config3_certified(team_plan):
    """The 512 certified config-3 instances (every bin: 128 / 256 / 127 / 1 at NC 96 / 128 /
    160 / 192) as one team-mode batch, each replicated twice (1,024 instances: two teams per CU
    share the SIMDs)."""
    from cmpc import solve_batch, synth
    fx = load_fixture("qp_cfg3.npz")
    b = synth.make_config(3, B=65536)
    sub = {k: np.repeat(b[k][fx["idx"]], 2, axis=0) for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}
    w, st, it = solve_batch(sub, plan=team_plan)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    err = rel_err_U(w, np.repeat(fx["w"], 2, axis=0))
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()) // 2)


def test_team_matches_one_wave(team_plan, wave_plan):
    """Team and one-wave kernels on the same 2,048 mixed instances: both solve every instance,
    and their U agree to the parity bar (both are within 1e-4 of the same unique optimum)."""
    from cmpc import solve_batch, synth
    b = synth.make_config(2, B=2048)
    wt, st, it = solve_batch(b, plan=team_plan)
    ww, sw, iw = solve_batch(b, plan=wave_plan)
    assert np.all(st == 1) and np.all(sw == 1)
    assert rel_err_U(wt, ww).max() <= 2 * TOL_U
    # the mean iteration count is a property of the algorithm, not of the kernel
    assert abs(it.mean() - iw.mean()) < 1.0, (it.mean(), iw.mean())


def test_team_edge_patterns(team_plan):
    """All-swing (no free force), all-stance (192 free forces), single foot, alternating."""
    from cmpc import solve_batch, synth
    from oracle import mpc_qp, tight_solver
    b = synth.make_config(2, B=6)
    b["contact"][0] = 0
    b["contact"][1] = 1
    b["contact"][2] = 0
    b["contact"][2, 1] = 1
    b["contact"][3] = 0
    b["contact"][3, :, ::2] = 1
    w, st, it = solve_batch(b, plan=team_plan)
    assert np.all(st == 1), st
    Xg, Ug = split_w(w.astype(np.float64))
    assert np.all(Ug[0] == 0)
    for i in range(4):
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        assert rel_err_U(w[i:i + 1], tight_solver.solve(qp)["w"][None])[0] <= TOL_U


def test_team_deterministic(team_plan):
    from cmpc import solve_batch, synth
    b = synth.make_config(3, B=512)
    w1, s1, i1 = solve_batch(b, plan=team_plan)
    w2, s2, i2 = solve_batch(b, plan=team_plan)
    assert np.array_equal(w1, w2) and np.array_equal(s1, s2) and np.array_equal(i1, i2)


def test_team_multipliers_and_warm_start(team_plan):
    """cmpc_solve_ref in team mode: the reference's multipliers against the certified ones,
    then a warm start from the certified (w, lam) polishes directly (0 iterations); a park /
    restore of the inverse is exercised by the hard cases (failed polish sessions)."""
    from cmpc import to_device_batch
    fx = load_fixture("qp_cfg2.npz")
    d = to_device_batch(fixture_batch(fx), team_plan.device)
    w, st, it, lam = team_plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"],
                                     d["contact"], lam_out=True)
    torch.cuda.synchronize(team_plan.device)
    ref = np.concatenate([fx["lam_x"], fx["lam_a"]], axis=1)
    lam = lam.cpu().numpy().astype(np.float64)
    err = np.max(np.abs(lam - ref), 1) / np.maximum(np.max(np.abs(ref), 1), 1e-9)
    assert torch.all(st == 1) and err.max() <= TOL_U, err.max()
    f32 = torch.float32
    w0 = torch.as_tensor(fx["w"], dtype=f32, device=team_plan.device).contiguous()
    l0 = torch.as_tensor(ref, dtype=f32, device=team_plan.device).contiguous()
    w, st, it = team_plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                                w_init=w0, lam_init=l0)
    torch.cuda.synchronize(team_plan.device)
    assert torch.all(st == 1) and int(it.max()) == 0
    assert rel_err_U(w.cpu().numpy(), fx["w"]).max() <= TOL_U


def test_team_park_restore_paths(team_plan):
    """Hard instances (failed polish sessions: park, restore, refactor at rho0) replicated to
    256 teams each, against their certified optimum."""
    from cmpc import solve_batch
    fx = load_fixture("qp_hard.npz")
    reps = 256
    batch = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
    w, st, it = solve_batch(batch, plan=team_plan)
    assert np.all(st == 1)
    err = rel_err_U(w, np.repeat(fx["w"], reps, axis=0))
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()) // reps)


@pytest.mark.parametrize("name", ["qp_cfg1.npz", "qp_cfg2.npz", "qp_nc192.npz"])
def test_one_wave_latency_mode_parity(wave_plan, name):
    """With team mode off, small batches run one wave per QP in latency mode (block-row
    condensation for NC <= 128): same parity bar."""
    from cmpc import solve_batch
    fx = load_fixture(name)
    w, st, it = solve_batch(fixture_batch(fx), plan=wave_plan)
    assert np.all(st == 1), (st, it)
    err = rel_err_U(w, fx["w"])
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()))
