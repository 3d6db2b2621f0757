"""CPU: the C-ABI library loads, exports every symbol include/cmpc.h declares, and
validates parameters without touching a GPU."""
import ctypes
import re

import pytest

from conftest import REPO


def declared_symbols():
    h = (REPO / "include" / "cmpc.h").read_text()
    return sorted(set(re.findall(r"\b(cmpc_[a-z_]+)\s*\(", h)))


@pytest.fixture(scope="module")
def lib():
    from cmpc import _lib
    from cmpc.build import build_library, LIB
    if not LIB.exists():
        build_library()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 8
    for s in syms:
        assert hasattr(lib, s), s
    from cmpc import _lib
    assert set(_lib.EXPORTS) <= set(syms)


def test_defaults_are_reference_constants(lib):
    from cmpc import _lib
    p = _lib.CParams()
    lib.cmpc_params_default(ctypes.byref(p))
    assert p.abi_version == _lib.ABI_VERSION and p.N == 16
    assert list(p.Q) == [1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1]        # centroidal_mpc.py:12
    assert all(abs(r - 1e-5) < 1e-12 for r in p.R)                       # :13
    assert abs(p.mu - 0.8) < 1e-7 and p.fz_min == 10.0                   # :15, :127
    assert abs(p.eps_abs - 1e-4) < 1e-9 and p.max_iter == 1000           # :25-27
    assert p.adaptive_rho_interval == 25                                 # :32
    assert p.reserved0 == 0  # ABI 4's ipm_facts (the interior-point fallback, removed in ABI 5)
    assert p.check_termination == 1  # OPTS check_termination (:31 has 10; include/cmpc.h says why)
    assert ctypes.sizeof(_lib.CParams) == 176  # include/cmpc.h layout (int64 max_batch at 168)
    assert _lib.CParams.max_batch.offset == 168
    assert lib.cmpc_version().decode().startswith("cmpc 1")


@pytest.mark.parametrize("field,value", [("N", 0), ("N", 17), ("mu", -1.0), ("max_iter", 0),
                                         ("alpha", 2.5), ("rho", 0.0), ("max_batch", 0),
                                         ("reserved0", 8), ("reserved0", -1),
                                         ("check_termination", 0), ("abi_version", 4)])
def test_invalid_params_rejected_before_device(lib, field, value):
    from cmpc import _lib
    p = _lib.CParams()
    lib.cmpc_params_default(ctypes.byref(p))
    setattr(p, field, value)
    h = ctypes.c_void_p()
    rc = lib.cmpc_plan_create(ctypes.byref(p), ctypes.byref(h))
    assert rc == -22
    assert "cmpc_plan_create" in lib.cmpc_last_error().decode()


def test_library_has_no_interior_point_fallback(lib):
    """ABI 5: the interior-point fallback and its controls are gone from the library (an ABI-4
    caller's ipm_facts > 0 is rejected as reserved0 before the device)."""
    assert not hasattr(lib, "cmpc_plan_set_ipm") and not hasattr(lib, "cmpc_plan_ipm_batch")
    from cmpc import _lib
    p = _lib.CParams()
    lib.cmpc_params_default(ctypes.byref(p))
    p.reserved0 = 8
    h = ctypes.c_void_p()
    assert lib.cmpc_plan_create(ctypes.byref(p), ctypes.byref(h)) == -22
    assert "reserved0" in lib.cmpc_last_error().decode()


def test_null_arguments(lib):
    assert lib.cmpc_plan_create(None, None) == -22
    assert lib.cmpc_solve(None, 1, *([None] * 10)) == -22
    assert lib.cmpc_plan_set_timing(None, 1) == -22
    assert lib.cmpc_build_dynamics(None, 1, 0.02, *([None] * 8)) == -22
    assert "cmpc_build_dynamics" in lib.cmpc_last_error().decode()
    assert lib.cmpc_solve_warm(None, 1, *([None] * 13)) == -22
    assert "cmpc_solve_warm" in lib.cmpc_last_error().decode()
    assert lib.cmpc_generate_traj(None, 1, 0.02, *([None] * 11)) == -22
    assert "cmpc_generate_traj" in lib.cmpc_last_error().decode()
    assert lib.cmpc_leg_torque(None, 1, None, None, None, 12, *([None] * 12), 45.0, None, None) == -22
    assert "cmpc_leg_torque" in lib.cmpc_last_error().decode()
    assert lib.cmpc_srb_step(None, 1, 20, 0.001, *([None] * 5), 12, *([None] * 5)) == -22
    assert "cmpc_srb_step" in lib.cmpc_last_error().decode()
    for name in ("cmpc_plan_set_team", "cmpc_plan_set_heavy_first"):
        assert getattr(lib, name)(None, -1) == -22
        assert name in lib.cmpc_last_error().decode()
    assert lib.cmpc_plan_heavy_first_batch(None, None) == -22
    assert lib.cmpc_plan_stats(None, None, 0) == -22
    assert "cmpc_plan_stats" in lib.cmpc_last_error().decode()
    lib.cmpc_plan_destroy(None)


def test_python_params_roundtrip():
    from cmpc import SolverParams
    c = SolverParams(N=12, mu=0.6, max_batch=7).to_c()
    assert c.N == 12 and abs(c.mu - 0.6) < 1e-7 and c.max_batch == 7
    with pytest.raises(ValueError):
        SolverParams(Q=(1, 2)).to_c()


def test_no_cpu_fallback_without_device():
    import torch
    from cmpc import Plan, CmpcError
    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(CmpcError):
        Plan()
