"""CPU: the oracle (oracle/) against the reference's own outputs and invariants.

ref_inputs.npz was produced by running the reference's gait.py / com_trajectory.py;
qp_assembly.npz by running the reference's CentroidalMPC QP assembly (centroidal_mpc.py:41-67,
122-359) unmodified under a conversion-only casadi stand-in (tests/golden/make_golden.py,
tests/golden/casadi_standin.py); the QP fixtures hold KKT-certified optima.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import mpc_qp, tight_solver
from cmpc import synth
from parity_util import load_fixture, fixture_batch


def _cases():
    z = load_fixture("ref_inputs.npz")
    n = int(z["n_cases"])
    return [{k[len(f"c{i}_"):]: v for k, v in z.items() if k.startswith(f"c{i}_")} for i in range(n)]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"hz{c['hz']}_duty{c['duty']}")
def test_contact_table_matches_reference(case):
    N = int(case["N"])
    ct = mpc_qp.contact_table(float(case["t_now"]), float(case["dt"]), N, float(case["hz"]),
                              float(case["duty"]))
    assert np.array_equal(ct, case["contact"])
    ct2 = synth.contact_table(float(case["t_now"]), float(case["dt"]), N, float(case["hz"]),
                              float(case["duty"]))
    assert np.array_equal(ct2.astype(np.int32), case["contact"])


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"hz{c['hz']}_duty{c['duty']}")
def test_dynamics_match_reference(case):
    r_legs = case["r_legs"]                       # (N, 4, 3)
    Ac, Bc, gc = mpc_qp.continuous_dynamics(float(case["m"]), case["I"], r_legs,
                                            float(case["yaw_avg"]))
    assert np.allclose(Ac, case["Ac"], atol=1e-14)
    assert np.allclose(Bc, case["Bc"], atol=1e-12)
    assert np.allclose(gc, case["gc"])
    Ad, Bd, gd = mpc_qp.discrete_dynamics(Ac, Bc, gc, float(case["dt"]))
    assert np.allclose(Ad, case["Ad"], atol=1e-13)
    assert np.allclose(Bd, case["Bd"], atol=1e-13)
    assert np.allclose(gd, case["gd"], atol=1e-13)
    Ad2, Bd2, gd2 = mpc_qp.discrete_dynamics_closed_form(Ac, Bc, gc, float(case["dt"]))
    assert np.allclose(Ad2, case["Ad"], atol=1e-13)
    assert np.allclose(Bd2, case["Bd"], atol=1e-13)
    assert np.allclose(gd2, case["gd"], atol=1e-13)
    # the product-side batched generator uses the same closed form
    Ad3, Bd3, gd3 = synth.discretize(np.array([case["m"]]), case["I"][None], r_legs[None],
                                     np.array([case["yaw_avg"]]), float(case["dt"]))
    assert np.allclose(Ad3[0], case["Ad"], atol=1e-13)
    assert np.allclose(Bd3[0], case["Bd"], atol=1e-13)
    assert np.allclose(gd3[0], case["gd"], atol=1e-13)


def test_qp_structure_matches_reference_print():
    """centroidal_mpc.py:225-230 invariants: H 384x384 nnz 384; A 448x384 nnz 5168 (0.0300)."""
    b = synth.make_config(1, B=1)
    qp = mpc_qp.build_qp(b["Ad"][0], b["Bd"][0], b["gd"][0], b["x0"][0], b["xref"][0].T,
                         b["contact"][0])
    assert qp["h"].shape == (384, 384) and qp["h"].nnz == 384
    assert qp["a"].shape == (448, 384) and qp["a"].nnz == 5168 == mpc_qp.structural_nnz(16)
    assert round(5168 / (448 * 384), 4) == 0.0300
    assert qp["lba"].shape == (448,) and qp["lbx"].shape == (384,)


@pytest.mark.parametrize("name", ["qp_cfg1.npz", "qp_cfg2.npz", "qp_hard.npz", "qp_nc192.npz"])
def test_golden_fixtures_are_kkt_certified(name):
    fx = load_fixture(name)
    n = fx["w"].shape[0]
    for i in range(0, n, 8 if n > 8 else 1):
        qp = mpc_qp.build_qp(fx["Ad"][i], fx["Bd"][i], fx["gd"][i], fx["x0"][i], fx["xref"][i].T,
                             fx["contact"][i])
        k = mpc_qp.kkt_residuals(qp, fx["w"][i], fx["lam_x"][i], fx["lam_a"][i])
        assert max(k.values()) < 1e-8, (i, k)


def test_tight_solver_certifies_fresh_instance():
    b = synth.make_config(2, B=3)
    qp = mpc_qp.build_qp(b["Ad"][2], b["Bd"][2], b["gd"][2], b["x0"][2], b["xref"][2].T,
                         b["contact"][2])
    r = tight_solver.solve(qp)
    assert max(r["kkt"].values()) < 1e-8


def test_rollout_matches_equality_rows():
    fx = load_fixture("qp_cfg1.npz")
    X, U = mpc_qp.unpack_w(fx["w"][0])
    Xr = mpc_qp.rollout(fx["Ad"][0], fx["Bd"][0], fx["gd"][0], fx["x0"][0], U.T)
    assert np.allclose(Xr.T, X, atol=1e-9)


def test_duals_recovered_from_primal():
    """cmpc.duals (host post-processing of the single-robot API) reproduces the certified
    multipliers from the certified primal."""
    from cmpc import duals
    fx = load_fixture("qp_cfg2.npz")
    for i in range(4):
        lx, la = duals.recover(fx["Ad"][i], fx["Bd"][i], fx["gd"][i], fx["x0"][i], fx["xref"][i],
                               fx["contact"][i], fx["w"][i], mpc_qp.Q_DIAG, mpc_qp.R_DIAG,
                               mpc_qp.MU, mpc_qp.FZ_MIN)
        scale = max(1e-3, np.max(np.abs(fx["lam_a"][i])))
        assert np.max(np.abs(la - fx["lam_a"][i])) < 1e-6 * scale + 1e-9
        assert np.max(np.abs(lx - fx["lam_x"][i])) < 1e-6 * scale + 1e-9


# ---- the QP assembly against the reference's own CentroidalMPC (qp_assembly.npz) ----------
def _assembly():
    return load_fixture("qp_assembly.npz")


def _ref_A(asm, j):
    shape = tuple(int(x) for x in asm["A_shape"])
    return sp.csc_matrix((asm["A_vals"][j], asm["A_row"], asm["A_colind"]), shape=shape)


def _fixture_instance(src):
    names = ("qp_cfg1.npz", "qp_cfg2.npz", "qp_hard.npz")
    fx = load_fixture(names[int(src[0])])
    return fx, int(src[1])


def test_reference_init_print_structure():
    """The reference's own __init__ / _build_sparse_matrix print (centroidal_mpc.py:225-230),
    captured when make_golden ran it: H 384 x 384 nnz 384, A 448 x 384 nnz 5168."""
    txt = str(_assembly()["init_print"])
    assert "H:  384 x 384  | nnz =    384" in txt
    assert "A:  448 x 384  | nnz =   5168 | dens =  0.0300" in txt
    assert "constr: 448 | horizon N = 16" in txt


def test_qp_assembly_vectors_match_reference_run():
    """g, lba, uba (_update_sparse_matrix, :235-285) and lbx, ubx (_compute_bounds, :122-176)
    from the reference's own code equal oracle.mpc_qp.build_qp on all 100 fixture instances."""
    asm = _assembly()
    n = asm["g"].shape[0]
    assert n == 100
    for j in range(n):
        fx, i = _fixture_instance(asm["src"][j])
        qp = mpc_qp.build_qp(fx["Ad"][i], fx["Bd"][i], fx["gd"][i], fx["x0"][i], fx["xref"][i].T,
                             fx["contact"][i])
        for key in ("g", "lba", "uba", "lbx", "ubx"):
            ref, mine = asm[key][j], qp[key]
            fin = np.isfinite(ref)
            assert np.array_equal(fin, np.isfinite(mine)), (j, key)
            assert np.array_equal(ref[~fin], mine[~fin]), (j, key)
            scale = max(1.0, float(np.max(np.abs(ref[fin])))) if fin.any() else 1.0
            assert np.max(np.abs(ref[fin] - mine[fin]), initial=0.0) <= 1e-14 * scale, (j, key)
        assert np.array_equal(asm["H"], qp["h"].toarray())


def test_qp_assembly_matrix_matches_reference_run():
    """A (_assemble_A_matrix + _precompute_friction_matrix + the SX dyn_builder,
    :287-359): the reference's structural pattern (5168 entries) and values equal the oracle's."""
    asm = _assembly()
    for j in range(asm["A_vals"].shape[0]):
        fx, i = _fixture_instance(asm["src"][j])
        Aref = _ref_A(asm, j)
        Aor = mpc_qp.constraint_matrix(fx["Ad"][i], fx["Bd"][i])
        assert Aref.nnz == Aor.nnz == 5168
        Aor_c = Aor.tocoo()
        po = set(zip(Aor_c.row.tolist(), Aor_c.col.tolist()))
        Aref_c = Aref.tocoo()
        assert po == set(zip(Aref_c.row.tolist(), Aref_c.col.tolist()))
        assert np.max(np.abs(Aref.toarray() - Aor.toarray())) <= 1e-15


def test_certified_optimum_is_the_reference_qps_optimum():
    """The golden primal/dual pairs are KKT points of the QP the REFERENCE assembled (not only
    of the oracle's restatement): with H, g, A, lba, uba, lbx, ubx from the reference run,
    stationarity / feasibility / complementarity hold to 1e-8.  The QP is strictly convex, so
    this pins the parity target to the reference's own problem."""
    asm = _assembly()
    for j in range(asm["A_vals"].shape[0]):
        fx, i = _fixture_instance(asm["src"][j])
        qp = dict(h=sp.csc_matrix(asm["H"]), a=_ref_A(asm, j), g=asm["g"][j], lba=asm["lba"][j],
                  uba=asm["uba"][j], lbx=asm["lbx"][j], ubx=asm["ubx"][j])
        k = mpc_qp.kkt_residuals(qp, fx["w"][i], fx["lam_x"][i], fx["lam_a"][i])
        assert max(k.values()) < 1e-8, (j, k)


def test_cfg3_fixture_is_kkt_certified():
    """qp_cfg3.npz stores indices into the config-3 generator: the digest matches and a sample
    of the stored optima are KKT points of the regenerated instances."""
    from parity_util import input_digest
    fx = load_fixture("qp_cfg3.npz")
    b = synth.make_config(3, B=65536)
    assert input_digest(b, fx["idx"]) == str(fx["digest"])
    for j in range(0, len(fx["idx"]), 32):
        i = int(fx["idx"][j])
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        k = mpc_qp.kkt_residuals(qp, fx["w"][j], fx["lam_x"][j], fx["lam_a"][j])
        assert max(k.values()) < 1e-8, (i, k)


def test_active_set_certifier_agrees_with_the_fixtures():
    """oracle/active_set.py (the fast certifier used on whole GPU batches) returns the fixtures'
    certified optimum from the fixture's own answer (no step), from a seed that holds a wrong
    face (instance 3458 of test_warm_next_tick's batch: fy held at mu fz where the optimum is
    7.97 N -- the active-set step drops it) and from nothing (fallback to tight_solver)."""
    from oracle import active_set
    fx = load_fixture("qp_cfg2.npz")
    for i in range(0, 64, 8):
        qp = mpc_qp.build_qp(fx["Ad"][i], fx["Bd"][i], fx["gd"][i], fx["x0"][i], fx["xref"][i].T,
                             fx["contact"][i])
        r = active_set.certified_optimum(qp, fx["w"][i])
        assert r["steps"] == 0 and max(r["kkt"].values()) <= active_set.CERT_TOL
        assert np.max(np.abs(r["w"] - fx["w"][i])) <= 1e-6 * np.max(np.abs(fx["w"][i]))
    hb = synth.make_config(2, B=4096)
    rng = np.random.default_rng(5)
    x0 = hb["x0"] + rng.normal(scale=[2e-3] * 6 + [2e-2] * 6, size=hb["x0"].shape)
    i = 3458
    qp = mpc_qp.build_qp(hb["Ad"][i], hb["Bd"][i], hb["gd"][i], x0[i], hb["xref"][i].T,
                         hb["contact"][i])
    opt = tight_solver.solve(qp)
    seed = opt["w"].copy()
    seed[192 + 12 * 9 + 3 * 3 + 1] = 8.0          # step 9, leg RR: fy on the face mu fz
    r = active_set.certified_optimum(qp, seed)
    assert r["steps"] >= 1 and not r["fallback"]
    assert np.max(np.abs(r["w"] - opt["w"])) <= 1e-9 * np.max(np.abs(opt["w"]))
    r0 = active_set.certified_optimum(qp, np.zeros(384))
    assert max(r0["kkt"].values()) <= active_set.CERT_TOL
    assert np.max(np.abs(r0["w"] - opt["w"])) <= 1e-6 * np.max(np.abs(opt["w"]))


def test_next_tick_fixture_is_kkt_certified():
    """qp_next_tick.npz (test_warm_next_tick's certified subset): the digest matches the
    regenerated batch, the named round-4 near-misses carry KKT-certified (w, lam_x, lam_a), and a
    sample of the stored fp32 optima are the certified optima of their instances."""
    from oracle import active_set
    from parity_util import input_digest
    fx = load_fixture("qp_next_tick.npz")
    b = synth.next_tick(synth.make_config(2, B=4096))
    assert input_digest(b, fx["idx"]) == str(fx["digest"])
    assert len(fx["idx"]) >= 1024 and set(fx["named"]) <= set(fx["idx"])
    for j, i in enumerate(fx["named"]):
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        k = mpc_qp.kkt_residuals(qp, fx["named_w"][j], fx["named_lam_x"][j], fx["named_lam_a"][j])
        assert max(k.values()) < 1e-8, (i, k)
    for j in range(0, len(fx["idx"]), 97):
        i = int(fx["idx"][j])
        qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                             b["contact"][i])
        U = fx["U"][j].astype(np.float64)
        X = mpc_qp.rollout(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], U.reshape(16, 12))
        r = active_set.certified_optimum(qp, np.concatenate([X.reshape(-1), U]))
        assert max(r["kkt"].values()) <= active_set.CERT_TOL
        assert np.max(np.abs(r["w"][192:] - U)) <= 1e-6 * np.max(np.abs(U)), i
