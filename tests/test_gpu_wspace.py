"""GPU: the wrench-space factorization (csrc/cmpc_wspace.hip, every batch above the small-batch
bound) against the n-space kernels it replaced and the KKT-certified optimum, and the hand-off of
instances whose Bd is not of the centroidal form (com_trajectory.py:221-286) to the n-space
kernels.  Tolerance as in test_gpu_parity.py: max |U - U*| / max |U*| <= 1e-4."""
import os

import numpy as np
import pytest

from parity_util import load_fixture, fixture_batch, rel_err_U, split_w, rollout64, feasibility

pytestmark = pytest.mark.gpu
TOL_U = 1e-4


def _nspace_plan(**kw):
    """A plan whose large batches run the n-space kernels (CMPC_SOLVE_KERNEL=group)."""
    from cmpc import Plan, SolverParams
    old = os.environ.get("CMPC_SOLVE_KERNEL")
    os.environ["CMPC_SOLVE_KERNEL"] = "group"
    try:
        p = Plan(SolverParams(max_batch=65536, **kw))
    finally:
        if old is None:
            del os.environ["CMPC_SOLVE_KERNEL"]
        else:
            os.environ["CMPC_SOLVE_KERNEL"] = old
    assert p.solve_kernels(8192)[0].startswith("solve_group_kernel")
    return p


def test_large_batches_use_the_wrench_space_kernel(plan):
    assert plan.solve_kernels(8192)[0].startswith("solve_ws_kernel")
    assert plan.solve_kernels(65536) == ["solve_ws_kernel<false>", None]
    assert plan.solve_kernels(256)[0] == "solve_team_kernel<4>"


@pytest.mark.parametrize("cfg,B", [(3, 8192), (2, 4096)])
def test_agrees_with_nspace_kernels(plan, cfg, B):
    """Same solutions as the n-space path (both within the bar of the optimum) on a benchmark
    batch; every instance solved, feasible, X the rollout of U."""
    from cmpc import solve_batch, synth
    b = synth.make_config(cfg, B=B)
    w, st, it = solve_batch(b, plan=plan)
    w0, st0, _ = solve_batch(b, plan=_nspace_plan())
    assert np.all(st == 1) and np.all(st0 == 1), (np.unique(st), np.unique(st0))
    assert rel_err_U(w, w0).max() <= 2 * TOL_U
    Xg, Ug = split_w(w.astype(np.float64))
    assert feasibility(b, Ug).max() < 1e-2
    assert np.max(np.abs(Xg - rollout64(b, Ug))) < 1e-3


def test_unstructured_bd_handed_to_nspace_kernels(plan):
    """Instances whose Bd rows 0-5 are not 1/2 Ad[0:6, 6:12] Bd[6:12] (not the reference's
    discretisation) are solved by the n-space kernels after the wrench-space kernel: the
    structured copies match their certified optimum, the perturbed ones the certified optimum of
    THEIR QP (oracle/tight_solver.py), not the structure-projected one."""
    from cmpc import solve_batch
    from oracle import mpc_qp, tight_solver
    fx = load_fixture("qp_cfg2.npz")
    reps = 40
    b = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
    B = b["Ad"].shape[0]
    rng = np.random.default_rng(7)
    pert = np.zeros(B, bool)
    pert[1::reps] = True                     # one perturbed copy of every fixture instance
    Bd = b["Bd"].copy()
    noise = rng.standard_normal(Bd[pert][:, :, 0:6, :].shape).astype(np.float32)
    Bd[pert, :, 0:6, :] *= 1 + 0.05 * noise
    b["Bd"] = Bd
    w, st, it = solve_batch(b, plan=plan)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    keep = ~pert
    err = rel_err_U(w[keep], np.repeat(fx["w"], reps, axis=0)[keep])
    assert err.max() <= TOL_U, err.max()
    idx = np.flatnonzero(pert)[:4]
    for i in idx:
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        ref = tight_solver.solve(qp)["w"]
        assert rel_err_U(w[i:i + 1], ref[None])[0] <= TOL_U
        # (the perturbation is large enough to move the optimum: not the unperturbed answer)
        assert rel_err_U(w[i:i + 1], fx["w"][i // reps][None])[0] > 10 * TOL_U
