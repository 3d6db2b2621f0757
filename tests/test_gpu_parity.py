"""GPU parity: the HIP solver vs the KKT-certified float64 optimum (oracle/tight_solver.py)
on the committed fixtures, plus size-independent properties at the benchmark sizes.

Tolerance (BASELINE.json north_star): contact-force primal within 1e-4 relative,
max_k,leg |U_gpu - U*| / max |U*| <= 1e-4 per instance.
"""
import numpy as np
import pytest
import torch

from parity_util import (load_fixture, fixture_batch, rel_err_U, split_w, rollout64,
                         feasibility)

pytestmark = pytest.mark.gpu
TOL_U = 1e-4


@pytest.mark.parametrize("name", ["qp_cfg1.npz", "qp_cfg2.npz"])
def test_fixture_parity(plan, name):
    from cmpc import solve_batch
    fx = load_fixture(name)
    batch = fixture_batch(fx)
    w, st, it = solve_batch(batch, plan=plan)
    err = rel_err_U(w, fx["w"])
    assert np.all(st == 1), (st, it)
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()))
    # X is the rollout of U under the same dynamics (the equality rows of the reference QP)
    Xg, Ug = split_w(w.astype(np.float64))
    Xr = rollout64(batch, Ug)
    assert np.max(np.abs(Xg - Xr)) < 1e-4
    assert feasibility(batch, Ug).max() < 1e-3


def test_hard_cases(plan):
    """Benchmark-batch instances that exposed solver weaknesses (tests/golden/make_golden.py
    HARD_CASES: a degenerate vertex, an ill-conditioned face set, wandering repairs), each
    replicated past the latency-mode threshold (B > 4 x CUs) so they run the same arithmetic
    as in the 65,536-instance batch they came from."""
    from cmpc import solve_batch
    fx = load_fixture("qp_hard.npz")
    reps = 1100
    batch = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
    w, st, it = solve_batch(batch, plan=plan)
    assert np.all(st == 1), [(tuple(c), np.unique(st[i * reps:(i + 1) * reps]).tolist())
                             for i, c in enumerate(fx["cases"])]
    err = rel_err_U(w, np.repeat(fx["w"], reps, axis=0))
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()) // reps)
    assert it.max() < 400, [int(it[i * reps:(i + 1) * reps].max()) for i in range(len(fx["w"]))]


def test_status_and_iters_sane(plan):
    from cmpc import solve_batch, synth
    b = synth.make_config(2, B=4096)
    w, st, it = solve_batch(b, plan=plan)
    assert np.all(np.isfinite(w))
    assert np.mean(st == 1) > 0.99, np.unique(st, return_counts=True)
    Xg, Ug = split_w(w.astype(np.float64))
    assert feasibility(b, Ug).max() < 1e-2
    assert np.max(np.abs(Xg - rollout64(b, Ug))) < 1e-3


def _tight(batch, i):
    from oracle import mpc_qp, tight_solver
    qp = mpc_qp.build_qp(batch["Ad"][i], batch["Bd"][i], batch["gd"][i], batch["x0"][i],
                         batch["xref"][i].T, batch["contact"][i])
    r = tight_solver.solve(qp)
    assert max(r["kkt"].values()) < 1e-8
    return r["w"]


def test_edge_contact_patterns(plan):
    """All-swing (no free force), all-stance (192 free forces, largest bin), single foot."""
    from cmpc import solve_batch, synth
    b = synth.make_config(2, B=6)
    b["contact"][0] = 0
    b["contact"][1] = 1
    b["contact"][2] = 0
    b["contact"][2, 1] = 1
    b["contact"][3] = 0
    b["contact"][3, :, ::2] = 1
    w, st, it = solve_batch(b, plan=plan)
    assert np.all(st == 1), st
    Xg, Ug = split_w(w.astype(np.float64))
    assert np.all(Ug[0] == 0)
    assert np.max(np.abs(Xg[0] - rollout64(b, Ug)[0])) < 1e-4
    for i in range(4):
        wr = _tight(b, i)
        assert rel_err_U(w[i:i + 1], wr[None])[0] <= TOL_U


def test_shorter_horizon_plan():
    from cmpc import Plan, SolverParams, solve_batch, synth
    p = Plan(SolverParams(N=8, max_batch=16))
    b = synth.make_batch(5, seed=11, mixed=True, N=8)
    w, st, it = solve_batch(b, plan=p)
    assert w.shape == (5, 24 * 8) and np.all(st == 1)
    for i in range(5):
        assert rel_err_U(w[i:i + 1], _tight(b, i)[None], N=8)[0] <= TOL_U


def test_deterministic(plan):
    from cmpc import solve_batch, synth
    b = synth.make_config(2, B=512)
    w1, s1, i1 = solve_batch(b, plan=plan)
    w2, s2, i2 = solve_batch(b, plan=plan)
    assert np.array_equal(w1, w2) and np.array_equal(s1, s2) and np.array_equal(i1, i2)


def test_full_size_kkt_certificate(plan):
    """Config-3 sized batch (65,536 trot + mixed): every instance feasible, X consistent, and a
    float64 KKT certificate (multipliers recovered from the GPU primal) on a sample."""
    from cmpc import solve_batch, synth, duals
    from oracle import mpc_qp
    b = synth.make_config(3, B=65536)
    w, st, it = solve_batch(b, plan=plan)
    assert np.all(np.isfinite(w))
    solved = np.mean(st == 1)
    assert solved > 0.999, np.unique(st, return_counts=True)
    Xg, Ug = split_w(w.astype(np.float64))
    assert feasibility(b, Ug).max() < 1e-2
    rng = np.random.default_rng(0)
    for i in rng.choice(np.nonzero(st == 1)[0], 24, replace=False):
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        lx, la = duals.recover(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i],
                               b["contact"][i], w[i].astype(np.float64), mpc_qp.Q_DIAG,
                               mpc_qp.R_DIAG, mpc_qp.MU, mpc_qp.FZ_MIN, tol=1e-5)
        k = mpc_qp.kkt_residuals(qp, w[i].astype(np.float64), lx, la)
        gscale = np.max(np.abs(qp["g"])) + 1.0
        assert k["prim"] < 1e-3, (i, k)
        assert k["stat"] < 1e-3 * gscale, (i, k)
