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


def test_status_and_iters_sane(plan):
    from cmpc import solve_batch, synth
    b = synth.make_config(2, B=4096)
    w, st, it = solve_batch(b, plan=plan)
    assert np.all(np.isfinite(w))
    assert np.mean(st == 1) > 0.99, np.unique(st, return_counts=True)
    Xg, Ug = split_w(w.astype(np.float64))
    assert feasibility(b, Ug).max() < 1e-2
    assert np.max(np.abs(Xg - rollout64(b, Ug))) < 1e-3
