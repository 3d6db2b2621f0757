"""CPU: oracle/osqp_ref.cpp (the reference's OSQP solve restated; the CPU baseline)."""
import numpy as np
import pytest

from parity_util import load_fixture, fixture_batch, rel_err_U


@pytest.fixture(scope="module")
def osqp():
    from oracle import osqp_ref
    osqp_ref.build()
    return osqp_ref


def test_reference_opts_terminate(osqp):
    fx = load_fixture("qp_cfg1.npz")
    b = {k: v[:4] for k, v in fixture_batch(fx).items()}
    r = osqp.solve_batch(b, threads=2)
    assert np.all(r["status"] == 1)
    assert np.all((r["iters"] >= 10) & (r["iters"] <= 1000))
    # OSQP at eps 1e-4 is loose on this ill-conditioned QP: far from the optimum in U
    e = rel_err_U(r["w"], fx["w"][:4])
    assert np.all(e < 0.5)


def test_tight_settings_converge_to_certified_optimum(osqp):
    fx = load_fixture("qp_cfg2.npz")
    b = {k: v[:3] for k, v in fixture_batch(fx).items()}
    s = osqp.default_settings()
    s.eps_abs = s.eps_rel = 1e-10
    s.max_iter = 400000
    r = osqp.solve_batch(b, threads=3, settings=s)
    assert np.all(r["status"] == 1)
    assert rel_err_U(r["w"], fx["w"][:3]).max() < 1e-4
