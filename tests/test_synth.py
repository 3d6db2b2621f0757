"""CPU: synthetic batch generator and the algorithm model."""
import numpy as np
import pytest

from cmpc import synth


def test_config_shapes_and_determinism():
    a = synth.make_config(1, B=8)
    b = synth.make_config(1, B=8)
    for k in ("Ad", "Bd", "gd", "x0", "xref", "contact"):
        assert np.array_equal(a[k], b[k])
    assert a["Bd"].shape == (8, 16, 12, 12) and a["contact"].shape == (8, 4, 16)
    # config 1: one shared trot table (gait.py:26-37 at t0 = 0), 10 stance steps per leg
    assert np.all(a["contact"] == a["contact"][0])
    assert np.all(a["contact"][0].sum(1) == 10)


def test_mixed_masks_have_a_stance_foot_every_step():
    c = synth.make_config(2, B=512)
    assert np.all(c["contact"].sum(1) >= 1)
    nf = 3 * c["contact"].reshape(512, -1).sum(1)
    assert nf.min() >= 48 and nf.max() <= 192


def test_config3_interleaves():
    c = synth.make_config(3, B=9)
    assert c["Ad"].shape[0] == 9


@pytest.mark.slow
def test_algorithm_model_reaches_parity():
    """tests/algo_spec.py (NumPy model of the kernel's algorithm) on fixture instances."""
    import algo_spec
    from parity_util import load_fixture, fixture_batch, rel_err_U
    fx = load_fixture("qp_cfg2.npz")
    for i in (0, 5):
        inst = {k: v[i] for k, v in fixture_batch(fx).items()}
        out = algo_spec.solve(inst, algo_spec.Params())
        assert out["status"] == 1
        w = np.concatenate([np.zeros(192), out["U"].reshape(-1)])
        assert rel_err_U(w[None], fx["w"][i:i + 1])[0] < 1e-4


def test_algorithm_model_face_downdates():
    """tests/algo_spec.py with the kernel's face downdates (cmpc_wave.hip face_downdate) and its
    fp32 sweep inverse: the same certified optima, and the pure face-adding repairs skip their
    factorization (hard fixture instances, which repair)."""
    import algo_spec
    from parity_util import load_fixture, fixture_batch, rel_err_U
    fx = load_fixture("qp_hard.npz")
    fb = fixture_batch(fx)
    dd_reps = 0
    facts = [0, 0]
    for i in range(len(fx["w"])):
        inst = {k: v[i] for k, v in fb.items()}
        base = algo_spec.solve(inst, algo_spec.Params(fp32_polish=True))
        out = algo_spec.solve(inst, algo_spec.Params(fp32_polish=True, downdate=True, dd_max=6))
        assert out["status"] == 1
        w = np.concatenate([np.zeros(192), out["U"].reshape(-1)])
        assert rel_err_U(w[None], fx["w"][i:i + 1])[0] < 1e-4
        dd_reps += out["dd_repairs"]
        facts[0] += base["fact"]
        facts[1] += out["fact"]
    assert dd_reps > 0 and facts[1] < facts[0], (dd_reps, facts)


def test_algorithm_model_bordered_repairs():
    """tests/algo_spec.py with the kernel's bordered repairs (cmpc_wave.hip border_build /
    border_apply: dropped base faces as new parameters, added faces as constraints, on the
    session's base inverse): the same certified optima on the hard fixture instances, with
    repairs that drop faces and no more factorizations than the downdates alone."""
    import algo_spec
    from parity_util import load_fixture, fixture_batch, rel_err_U
    fx = load_fixture("qp_hard.npz")
    fb = fixture_batch(fx)
    facts = [0, 0]
    borders = 0
    for i in range(len(fx["w"])):
        inst = {k: v[i] for k, v in fb.items()}
        dd = algo_spec.solve(inst, algo_spec.Params(fp32_polish=True, downdate=True, dd_max=6))
        out = algo_spec.solve(inst, algo_spec.Params(fp32_polish=True, border=5, border_extra=12))
        assert out["status"] == 1
        w = np.concatenate([np.zeros(192), out["U"].reshape(-1)])
        assert rel_err_U(w[None], fx["w"][i:i + 1])[0] < 1e-4
        borders += out.get("border_repairs", 0)
        facts[0] += dd["fact"]
        facts[1] += out["fact"]
    assert borders > 0 and facts[1] <= facts[0], (borders, facts)
