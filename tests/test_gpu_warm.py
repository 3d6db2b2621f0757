"""GPU: warm-started solves (cmpc_solve_warm).

The reference warm-starts every tick's OSQP solve with the previous tick's primal and duals
(centroidal_mpc.py:91-95, stored at :108-110).  The warm start changes where the iteration
starts, not the answer: every warm-started result is held to the same bar as a cold one
(U within 1e-4 of the KKT-certified optimum, or of the cold solve of the same problem), and
must not take more iterations on a problem it has already solved.
"""
import numpy as np
import pytest
import torch

from parity_util import load_fixture, fixture_batch, rel_err_U, split_w, rollout64, feasibility

pytestmark = pytest.mark.gpu
TOL_U = 1e-4


def _dev(batch, plan):
    from cmpc.solver import to_device_batch
    return to_device_batch(batch, plan.device)


def _solve(plan, d, **kw):
    r = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], **kw)
    torch.cuda.synchronize(plan.device)
    return r


def test_warm_restart_at_the_optimum(plan):
    """Warm data = this problem's own solution and dual: the warm face set is the optimal one,
    so the first (direct) polish succeeds without ADMM iterations, and U is unchanged."""
    fx = load_fixture("qp_cfg1.npz")
    d = _dev(fixture_batch(fx), plan)
    w, st, it, y = _solve(plan, d, y_out=True)
    assert np.all(st.cpu().numpy() == 1)
    w2, st2, it2, y2 = _solve(plan, d, w_init=w, y_init=y, y_out=True)
    st2, it2, it = st2.cpu().numpy(), it2.cpu().numpy(), it.cpu().numpy()
    assert np.all(st2 == 1), np.unique(st2, return_counts=True)
    assert rel_err_U(w2.cpu().numpy(), fx["w"]).max() <= TOL_U
    assert np.all(it2 <= it), (it2.max(), it.max())
    # the warm face set goes straight to the polish: no ADMM iteration at all
    assert np.mean(it2 == 0) > 0.99, np.unique(it2, return_counts=True)
    assert it2.mean() < it.mean()
    # the returned dual is a fixed point too (same face set, same multipliers); instances whose
    # optimum is interior have y ~ 0, so the scale is the batch's largest multiplier
    yn, y2n = y.cpu().numpy(), y2.cpu().numpy()
    assert np.max(np.abs(y2n - yn)) < 1e-2 * np.abs(yn).max()


def _project_pyramid(F, mu, fz_min):
    """Euclidean projection of (..., 3) forces onto {|fx|, |fy| <= mu fz, fz >= fz_min}
    (float64; the same case split as the solver's z-update)."""
    a, b, c = F[..., 0], F[..., 1], F[..., 2]
    A, Bb = np.abs(a), np.abs(b)
    lo, hi = np.minimum(A, Bb), np.maximum(A, Bb)
    z1 = (c + mu * (A + Bb)) / (1 + 2 * mu * mu)
    z2 = (c + mu * hi) / (1 + mu * mu)
    z = np.where(mu * z1 < lo, z1, np.where(mu * z2 < hi, z2, c))
    z = np.maximum(z, fz_min)
    lim = mu * z
    return np.stack([np.clip(a, -lim, lim), np.clip(b, -lim, lim), z], axis=-1)


def test_dual_out_is_a_kkt_multiplier(plan):
    """y_out: zero on swing legs; on stance legs y lies in the normal cone of the friction
    pyramid at u -- moving u along y and projecting back returns u (complementarity)."""
    from cmpc import synth
    b = synth.make_config(2, B=512)
    d = _dev(b, plan)
    w, st, it, y = _solve(plan, d, y_out=True)
    ok = st.cpu().numpy() == 1
    assert ok.mean() > 0.99
    _, U = split_w(w.cpu().numpy().astype(np.float64))
    Y = y.cpu().numpy().astype(np.float64)
    F = U.reshape(len(U), 16, 4, 3)
    L = Y.reshape(len(U), 16, 4, 3)
    ct = b["contact"].transpose(0, 2, 1).astype(bool)          # (B, N, 4)
    assert np.all(L[~ct] == 0)
    fmax = np.abs(U).reshape(len(U), -1).max(1)
    lmax = np.abs(Y).max()  # batch scale: an interior optimum has y ~ 0 (rounding only)
    t = (0.1 * fmax / lmax)[:, None, None, None]
    P = _project_pyramid(F + t * L, plan.params.mu, plan.params.fz_min)
    dev = np.where(ct[..., None], np.abs(P - F), 0.0).reshape(len(U), -1).max(1) / fmax
    assert dev[ok].max() < 1e-3, (dev[ok].max(), int(np.flatnonzero(ok)[dev[ok].argmax()]))


def _rel_err_fixture(w, U_opt):
    """max|dU| / max|U*| per instance against fp32-stored certified optima (B, 12N)."""
    Ug = np.asarray(w, np.float64)[:, 12 * 16:]
    Uo = np.asarray(U_opt, np.float64)
    return np.max(np.abs(Ug - Uo), axis=1) / np.maximum(np.max(np.abs(Uo), axis=1), 1e-12)


def test_warm_next_tick(plan):
    """Closed-loop proxy: the next tick's problem (state moved, same reference and gait;
    synth.next_tick) cold, warm-started from this tick's (w, y) as centroidal_mpc.py:91-95 does
    without shifting, and warm-started from this tick's REFERENCE multipliers (cmpc_solve_ref).
    Every instance of the committed certified subset (tests/golden/qp_next_tick.npz: 1,024 of the
    4,096 plus the four instances that exposed the fp32 check's flat-direction limit in round 4)
    must be status 1 and within 1e-4 of its certified optimum in all three solves, and the
    slowest warm instance takes no more ADMM iterations than the slowest cold one."""
    from cmpc import synth
    from parity_util import input_digest
    b = synth.make_config(2, B=4096)
    b2 = synth.next_tick(b)
    fx = load_fixture("qp_next_tick.npz")
    idx = fx["idx"]
    assert input_digest(b2, idx) == str(fx["digest"])
    d = _dev(b, plan)
    w, st, it, y = _solve(plan, d, y_out=True)
    w1, st1, it1, lam1 = _solve(plan, d, lam_out=True)
    d2 = _dev(b2, plan)
    wc, stc, itc = _solve(plan, d2)
    ww, stw, itw, yw = _solve(plan, d2, w_init=w, y_init=y, y_out=True)
    wr, str_, itr, _ = _solve(plan, d2, w_init=w1, lam_init=lam1, lam_out=True)
    for tag, wx, sx in (("cold", wc, stc), ("warm", ww, stw), ("warm ref", wr, str_)):
        sn = sx.cpu().numpy()
        assert np.all(sn[idx] == 1), (tag, np.unique(sn[idx], return_counts=True))
        err = _rel_err_fixture(wx.cpu().numpy()[idx], fx["U"])
        assert err.max() <= TOL_U, (tag, err.max(), int(idx[err.argmax()]))
        for i in fx["named"]:  # the round-4 near-misses by name
            assert err[np.searchsorted(idx, i)] <= TOL_U, (tag, int(i))
    stc, stw = stc.cpu().numpy(), stw.cpu().numpy()
    itc, itw = itc.cpu().numpy(), itw.cpu().numpy()
    assert np.mean(stw == 1) >= np.mean(stc == 1) - 1e-3
    assert np.mean(stc == 1) > 0.99 and np.mean(stw == 1) > 0.99
    assert itw.mean() < itc.mean(), (itw.mean(), itc.mean())
    assert np.mean(itw == 0) > 0.95, np.unique(itw, return_counts=True)
    # the warm tail is no worse than cold: a warm start whose face set fails its polish session
    # restarts as the cold solve (cmpc_wave.hip solve_instance, kWarmRestart)
    assert itw.max() <= itc.max(), (int(itw.max()), int(itc.max()), int(itw.argmax()))
    # every instance, not only the certified subset: where cold and warm both verified their
    # answer (status 1, each within 1e-4 of the same unique optimum), they agree within 2e-4
    both = (stc == 1) & (stw == 1)
    assert both.mean() > 0.99
    dcw = rel_err_U(ww.cpu().numpy()[both], wc.cpu().numpy()[both])
    assert dcw.max() <= 2 * TOL_U, (dcw.max(), int(np.flatnonzero(both)[dcw.argmax()]))
    Xg, Ug = split_w(ww.cpu().numpy().astype(np.float64))
    assert feasibility(b2, Ug).max() < 1e-2
    assert np.max(np.abs(Xg - rollout64(b2, Ug))) < 1e-3


def test_warm_garbage_and_aliasing(plan):
    """Non-finite / huge warm data and in-place warm buffers (w_init is w_out, y_init is
    y_out) still give the certified answer."""
    fx = load_fixture("qp_cfg1.npz")
    d = _dev(fixture_batch(fx), plan)
    B = d["Ad"].shape[0]
    g = torch.Generator(device="cpu").manual_seed(3)
    w = (torch.randn((B, 24 * 16), generator=g) * 1e3).to(plan.device)
    y = (torch.randn((B, 12 * 16), generator=g) * 1e2).to(plan.device)
    w[::7] = float("nan")
    y[::5] = float("inf")
    st = torch.empty((B,), dtype=torch.int32, device=plan.device)
    it = torch.empty_like(st)
    _solve(plan, d, out=(w, st, it), w_init=w, y_init=y, y_out=y)
    stn = st.cpu().numpy()
    assert np.mean(stn == 1) > 0.99, np.unique(stn, return_counts=True)
    ok = stn == 1
    assert rel_err_U(w.cpu().numpy()[ok], fx["w"][ok]).max() <= TOL_U
    assert torch.isfinite(y).all()


def test_warm_primal_only_and_dual_only(plan):
    fx = load_fixture("qp_cfg1.npz")
    d = _dev(fixture_batch(fx), plan)
    w, st, it, y = _solve(plan, d, y_out=True)
    for kw in (dict(w_init=w), dict(y_init=y)):
        w2, st2, it2 = _solve(plan, d, **kw)
        assert np.all(st2.cpu().numpy() == 1)
        assert rel_err_U(w2.cpu().numpy(), fx["w"]).max() <= TOL_U


# Fresh-seed warm tick (round 6, profiles/r06s_*, r06v_*): instances 31439 and 5794 of
# synth.next_tick(make_batch(65536, 13, mixed)) warm from the previous tick are accepted at the
# default polish_refine 2 with 2.1e-4 / 1.1e-4 error along directions weighed only by R
# (DESIGN.md 8); polish_refine 4 brings them within the bar.  Each instance is solved
# independently of the others (test_instance_order_independent), so the two, replicated past the
# team bound (the one-wave kernels of the 65,536 batch), reproduce their in-batch answers.
_FRESH_IDS = (31439, 5794)


def _fresh_pair(reps=1100):
    from cmpc import synth
    prev = synth.make_batch(65536, 13, mixed=True)
    nxt = synth.next_tick(prev)
    keys = ("Ad", "Bd", "gd", "x0", "xref", "contact")
    ids = np.repeat(np.array(_FRESH_IDS), reps)
    return ({k: prev[k][ids] for k in keys}, {k: nxt[k][ids] for k in keys}, nxt)


def _fresh_errors(polish_refine):
    from cmpc import Plan, SolverParams
    from oracle import mpc_qp, tight_solver
    prev, nxt, full = _fresh_pair()
    p = Plan(SolverParams(max_batch=len(prev["x0"]), polish_refine=polish_refine))
    dp, dn = _dev(prev, p), _dev(nxt, p)
    w0, _, _, y0 = _solve(p, dp, y_out=True)
    w, st, it, _ = _solve(p, dn, w_init=w0, y_init=y0, y_out=True)
    w, st = w.cpu().numpy(), st.cpu().numpy()
    errs = []
    for j, i in enumerate(_FRESH_IDS):
        qp = mpc_qp.build_qp(full["Ad"][i], full["Bd"][i], full["gd"][i], full["x0"][i],
                             full["xref"][i].T, full["contact"][i])
        r = tight_solver.solve(qp)
        assert max(r["kkt"].values()) < 1e-8
        rows = slice(j * 1100, (j + 1) * 1100)
        errs.append((st[rows], rel_err_U(w[rows], np.repeat(r["w"][None], 1100, axis=0))))
    return errs


def test_fresh_warm_tick_strict_setting():
    """polish_refine 4: every status-1 answer of the two fresh-seed misses within 1e-4."""
    for st, err in _fresh_errors(4):
        assert np.all(err[st == 1] <= TOL_U), (np.unique(st), float(err.max()))


@pytest.mark.xfail(reason="known gap at the default polish_refine 2: R-weighted directions "
                          "(DESIGN.md 8)", strict=False)
def test_fresh_warm_tick_default_setting():
    for st, err in _fresh_errors(2):
        assert np.all(err[st == 1] <= TOL_U), (np.unique(st), float(err.max()))
