"""GPU: the reference's multipliers (lam_x, lam_a; centroidal_mpc.py:91-95, 108-110) produced
and consumed on the device by cmpc_solve_ref, against the KKT-certified float64 multipliers of
the fixtures (oracle/tight_solver.py, CasADi's sign convention).

The multipliers of this QP are unique (per leg at most three active rows with independent
gradients, independent dynamics rows), so they are compared entry by entry.  Tolerance:
max |lam_gpu - lam*| <= 1e-4 x max |lam*| per instance (the primal bar of the north star,
applied to the duals).
"""
import numpy as np
import pytest
import torch

from parity_util import load_fixture, fixture_batch, rel_err_U, assert_verified

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _solve_lam(plan, batch, **kw):
    from cmpc import to_device_batch
    d = to_device_batch(batch, plan.device)
    w, st, it, lam = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                                lam_out=True, **kw)
    torch.cuda.synchronize(plan.device)
    return (w.cpu().numpy().astype(np.float64), st.cpu().numpy(), it.cpu().numpy(),
            lam.cpu().numpy().astype(np.float64))


def _lam_err(lam, lam_x_ref, lam_a_ref, N=16):
    ref = np.concatenate([lam_x_ref, lam_a_ref], axis=1)
    scale = np.maximum(np.max(np.abs(ref), axis=1), 1e-9)
    return np.max(np.abs(lam - ref), axis=1) / scale


@pytest.mark.parametrize("name", ["qp_cfg1.npz", "qp_cfg2.npz", "qp_hard.npz", "qp_nc192.npz"])
def test_device_multipliers_match_certified(plan, name):
    from oracle import mpc_qp
    fx = load_fixture(name)
    batch = fixture_batch(fx)
    w, st, it, lam = _solve_lam(plan, batch)
    assert np.all(st == 1)
    err = _lam_err(lam, fx["lam_x"], fx["lam_a"])
    assert err.max() <= TOL, (err.max(), int(err.argmax()))
    for i in range(0, len(st), max(1, len(st) // 8)):   # and they are KKT multipliers of w
        qp = mpc_qp.build_qp(batch["Ad"][i], batch["Bd"][i], batch["gd"][i], batch["x0"][i],
                             batch["xref"][i].T, batch["contact"][i])
        k = mpc_qp.kkt_residuals(qp, w[i], lam[i, :384], lam[i, 384:])
        assert k["prim"] < 1e-3 and k["stat"] < 1e-3 * (1 + np.max(np.abs(qp["g"]))), (i, k)


def test_device_multipliers_full_batch_sample(plan):
    """Config-3 batch (65,536): the multipliers of the 512 certified instances (every bin)."""
    from cmpc import synth
    fx = load_fixture("qp_cfg3.npz")
    b = synth.make_config(3, B=65536)
    w, st, it, lam = _solve_lam(plan, b)
    idx = fx["idx"]
    ok = assert_verified(st)
    err = np.where(ok[idx], _lam_err(lam[idx], fx["lam_x"], fx["lam_a"]), 0.0)
    assert err.max() <= TOL, (err.max(), int(idx[err.argmax()]))


def test_warm_start_from_reference_multipliers(plan):
    """The reference's warm start (x0 = previous w, lam_x0 / lam_a0 = previous multipliers):
    at the certified optimum the warm face set polishes directly (0 ADMM iterations) and the
    solution and multipliers are unchanged; dual-only warm starts converge too; NaN duals are
    ignored."""
    from cmpc import to_device_batch
    fx = load_fixture("qp_cfg2.npz")
    batch = fixture_batch(fx)
    d = to_device_batch(batch, plan.device)
    B = d["Ad"].shape[0]
    f32 = torch.float32
    w0 = torch.as_tensor(fx["w"], dtype=f32, device=plan.device).contiguous()
    l0 = torch.as_tensor(np.concatenate([fx["lam_x"], fx["lam_a"]], 1), dtype=f32,
                         device=plan.device).contiguous()
    w, st, it, lam = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                                w_init=w0, lam_init=l0, lam_out=True)
    torch.cuda.synchronize(plan.device)
    assert torch.all(st == 1) and int(it.max()) == 0
    assert rel_err_U(w.cpu().numpy(), fx["w"]).max() <= TOL
    assert _lam_err(lam.cpu().numpy().astype(np.float64), fx["lam_x"], fx["lam_a"]).max() <= TOL
    # dual only
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                           lam_init=l0)
    assert torch.all(st == 1)
    assert rel_err_U(w.cpu().numpy(), fx["w"]).max() <= TOL
    # in place (lam_init aliases lam_out), with garbage in half of it
    lbuf = l0.clone()
    lbuf[: B // 2] = float("nan")
    w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                           w_init=w0, lam_init=lbuf, lam_out=lbuf)
    torch.cuda.synchronize(plan.device)
    assert torch.all(st == 1)
    assert rel_err_U(w.cpu().numpy(), fx["w"]).max() <= TOL
    assert _lam_err(lbuf.cpu().numpy().astype(np.float64), fx["lam_x"], fx["lam_a"]).max() <= TOL


def test_lam_and_y_are_exclusive(plan):
    from cmpc import to_device_batch, synth
    d = to_device_batch(synth.make_config(1, B=2), plan.device)
    with pytest.raises(ValueError):
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], lam_out=True,
                   y_out=True)
