"""GPU: on-device QP-data generation (cmpc_build_dynamics) against the
reference's own discrete dynamics (tests/golden/ref_inputs.npz, produced by the reference's
com_trajectory.py with scipy cont2discrete + expm/trapz) and against the batched closed form.

Tolerance: the inputs cross the boundary as fp32 (m, I_com, lever arms, yaw), the device then
evaluates the exact closed form in fp64 and rounds once to fp32.  Input rounding moves I^-1 [r]x
by a few fp32 ulps of the block scale, so an entry must lie within 4e-7 of the array's largest
magnitude plus one fp32 rounding of itself (the reference's expm leaves ~1e-17 where the exact
value is 0)."""
import numpy as np
import pytest

from parity_util import load_fixture, fixture_batch

pytestmark = pytest.mark.gpu

REL = 2.0 ** -23  # one fp32 rounding of the exact value, with margin for the fp64 evaluation


def _close(gpu, ref):
    ref = np.asarray(ref, np.float64)
    err = np.abs(np.asarray(gpu, np.float64) - ref)
    ok = np.all(err <= REL * np.abs(ref) + 4e-7 * np.abs(ref).max() + 1e-12)
    if not ok:
        print("max err", err.max(), "scale", np.abs(ref).max())
    return ok


def _to_dev(a, torch):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32).cuda()


def test_golden_reference_dynamics(plan):
    import torch
    from conftest import REPO
    g = np.load(REPO / "tests" / "golden" / "ref_inputs.npz")
    for c in range(int(g["n_cases"])):
        p = f"c{c}_"
        N = int(g[p + "N"])
        assert N == plan.params.N
        xref = g[p + "xref"].T[None]                     # (1, N, 12): column k -> row k
        assert abs(xref[0, :, 5].mean() - float(g[p + "yaw_avg"])) < 1e-12  # :226 equivalence
        Ad, Bd, gd = plan.build_dynamics(_to_dev([g[p + "m"]], torch), _to_dev(g[p + "I"][None], torch),
                                         _to_dev(g[p + "r_legs"][None], torch), _to_dev(xref, torch),
                                         float(g[p + "dt"]))
        torch.cuda.synchronize()
        assert _close(Ad.cpu().numpy()[0], g[p + "Ad"]), c
        assert _close(Bd.cpu().numpy()[0], g[p + "Bd"]), c
        assert _close(gd.cpu().numpy()[0], g[p + "gd"]), c


def test_batched_closed_form_and_solve(plan):
    import torch
    from cmpc import synth, to_device_batch
    b = synth.make_config(3, B=4096)
    m, I, r, xr = (_to_dev(b[k], torch) for k in ("m", "I_world", "r_legs", "xref"))
    Ad, Bd, gd = plan.build_dynamics(m, I, r, xr, float(b["dt"]))
    torch.cuda.synchronize()
    assert _close(Ad.cpu().numpy(), b["Ad"])
    assert _close(Bd.cpu().numpy(), b["Bd"])
    assert _close(gd.cpu().numpy(), b["gd"])
    # the solve on device-built data matches the solve on host-built data
    d = to_device_batch(b)
    w0, s0, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
    w1, s1, _ = plan.solve(Ad, Bd, gd, d["x0"], d["xref"], d["contact"])
    torch.cuda.synchronize()
    s0, s1 = s0.cpu().numpy(), s1.cpu().numpy()
    assert np.mean(s1 == 1) > 0.999 and np.mean(s0 == 1) > 0.999
    U0 = w0.cpu().numpy()[:, 192:].astype(np.float64)
    U1 = w1.cpu().numpy()[:, 192:].astype(np.float64)
    ok = (s0 == 1) & (s1 == 1)
    rel = np.abs(U1 - U0).max(1) / np.maximum(np.abs(U0).max(1), 1.0)
    assert rel[ok].max() < 1e-4


def test_argument_validation(plan):
    import torch
    from cmpc import CmpcError
    z = torch.zeros(2, device="cuda")
    with pytest.raises((ValueError, CmpcError)):
        plan.build_dynamics(z, torch.zeros(2, 3, 3, device="cuda"),
                            torch.zeros(2, plan.params.N, 4, 3, device="cuda"),
                            torch.zeros(2, plan.params.N, 12, device="cuda"), -0.01)
