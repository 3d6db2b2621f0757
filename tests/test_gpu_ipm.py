"""GPU parity of the interior-point face-set identification (cmpc_wave.hip ipm_identify,
DESIGN.md 4h) against the KKT-certified optimum.

EXPERIMENTAL, variant build only: the default libcmpc.so does not carry the fallback (no
measured batch gains from it since the damped repairs).  Build and run it with
``bash scripts/build_variant.sh ipm -DCMPC_WITH_IPM`` and
``CMPC_LIB=convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_ipm.so pytest tests/test_gpu_ipm.py``;
with the default library these tests are skipped.

It is opt-in (cmpc_params.ipm_facts > 0; then on the hard instances of tail-bound batches,
B <= 64 x CUs, cmpc_plan_set_ipm).  These tests force it early (ipm_facts = 1: after the first
failed session)
so that every instance whose first polish session fails -- ~1-2 % of config 2 / 3 -- goes
through the interior-point steps, the polish session they start and, when that fails, the
restored ADMM state.  Tolerance as in test_gpu_parity.py: max |U - U*| / max |U*| <= 1e-4.
"""
import numpy as np
import pytest

from parity_util import load_fixture, fixture_batch, rel_err_U, split_w, rollout64, feasibility

pytestmark = pytest.mark.gpu
TOL_U = 1e-4


@pytest.fixture(scope="module")
def plan_ipm():
    from cmpc import Plan, SolverParams
    try:
        p = Plan(SolverParams(max_batch=65536, ipm_facts=1))
    except RuntimeError as e:
        if "CMPC_WITH_IPM" in str(e):
            pytest.skip("library built without the interior-point fallback (variant build only)")
        raise
    p.set_ipm(65536)  # the fallback-carrying kernels at every size (default: B <= 64 x CUs)
    return p


def test_hard_cases_forced(plan_ipm):
    """The four hard fixtures, replicated past the latency-mode threshold."""
    from cmpc import solve_batch
    fx = load_fixture("qp_hard.npz")
    reps = 1100
    batch = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
    w, st, it = solve_batch(batch, plan=plan_ipm)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    err = rel_err_U(w, np.repeat(fx["w"], reps, axis=0))
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()) // reps)


@pytest.mark.parametrize("name", ["qp_cfg2.npz", "qp_nc192.npz"])
def test_fixtures_forced(plan_ipm, name):
    from cmpc import solve_batch
    fx = load_fixture(name)
    reps = 40  # > 4 x CUs instances: the one-wave kernels (the team kernel has no fallback)
    batch = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
    w, st, it = solve_batch(batch, plan=plan_ipm)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    err = rel_err_U(w, np.repeat(fx["w"], reps, axis=0))
    assert err.max() <= TOL_U, (err.max(), int(err.argmax()) // reps)


def test_full_batch_forced(plan_ipm):
    """The whole config-3 batch with the fallback forced: every instance status 1, feasible, X
    the rollout of U, the 512 certified instances within 1e-4, and the same solutions as with
    the fallback off.  (Iteration counts are not compared: since the rho bump after the first
    failed session (cmpc_wave.hip kFailRho) the hard instances converge in fewer ADMM iterations
    without the fallback.)"""
    from cmpc import Plan, SolverParams, solve_batch, synth
    from parity_util import input_digest
    fx = load_fixture("qp_cfg3.npz")
    b = synth.make_config(3, B=65536)
    idx = fx["idx"]
    assert input_digest(b, idx) == str(fx["digest"]), "config-3 generator drifted"
    w, st, it = solve_batch(b, plan=plan_ipm)
    assert np.all(np.isfinite(w))
    assert np.all(st == 1), np.unique(st, return_counts=True)
    Xg, Ug = split_w(w.astype(np.float64))
    assert feasibility(b, Ug).max() < 1e-2
    sub = {k: b[k][idx] for k in ("Ad", "Bd", "gd", "x0")}
    assert np.max(np.abs(Xg[idx] - rollout64(sub, Ug[idx]))) < 1e-3
    err = rel_err_U(w[idx], fx["w"])
    assert err.max() <= TOL_U, (err.max(), int(idx[int(err.argmax())]))
    off = Plan(SolverParams(max_batch=65536, ipm_facts=0))
    off.set_ipm(65536)
    w0, st0, it0 = solve_batch(b, plan=off)
    assert np.all(st0 == 1)
    # both paths reach the same optimum (the fallback changes the route, not the answer)
    assert rel_err_U(w, w0).max() <= 2 * TOL_U
