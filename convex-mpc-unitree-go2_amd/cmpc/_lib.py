"""ctypes binding of the C-ABI declared in ``include/cmpc.h``.

This is the Python side of the drop-in boundary: the reference calls CasADi's conic/OSQP
plugin from Python (``centroidal_mpc.py:212-213, 98``); here Python calls ``libcmpc.so``.
The product path has no CPU fallback: if the library is missing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

from .build import LIB

ABI_VERSION = 6
# ABI 5 (round 5) has this cmpc_params layout, bins and solve kernels (it lacks cmpc_plan_stats
# and the certified status-1 bound): its builds load only for A/B experiments, with
# CMPC_ALLOW_ABI5=1
ABI_COMPAT = (5, 6) if os.environ.get("CMPC_ALLOW_ABI5") == "1" else (6,)
NUM_STATS = 4  # CMPC_NUM_STATS
CMPC_OK = 0


class CParams(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("N", ctypes.c_int32),
        ("Q", ctypes.c_float * 12),
        ("R", ctypes.c_float * 12),
        ("mu", ctypes.c_float),
        ("fz_min", ctypes.c_float),
        ("eps_abs", ctypes.c_float),
        ("eps_rel", ctypes.c_float),
        ("max_iter", ctypes.c_int32),
        ("rho", ctypes.c_float),
        ("sigma", ctypes.c_float),
        ("alpha", ctypes.c_float),
        ("adaptive_rho_interval", ctypes.c_int32),
        ("polish_stable", ctypes.c_int32),
        ("polish_refine", ctypes.c_int32),
        ("polish_tol", ctypes.c_float),
        ("polish_repairs", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("check_termination", ctypes.c_int32),
        ("max_batch", ctypes.c_int64),
    ]


EXPORTS = ("cmpc_params_default", "cmpc_plan_create", "cmpc_solve", "cmpc_plan_destroy",
           "cmpc_build_dynamics", "cmpc_solve_warm", "cmpc_solve_ref", "cmpc_generate_traj", "cmpc_leg_torque", "cmpc_srb_step",
           "cmpc_plan_set_timing", "cmpc_plan_timing_read", "cmpc_plan_set_team", "cmpc_plan_team_batch",
           "cmpc_plan_set_heavy_first",
           "cmpc_plan_heavy_first_batch", "cmpc_plan_solve_kernel", "cmpc_plan_stats",
           "cmpc_last_error", "cmpc_version")
NUM_BINS = 5
BIN_CAPS = (96, 128, 144, 160, 192)
# solve kernels (timing slots): 0 = bins NC 128 + 96 (two waves per SIMD), 1 = bins NC 160 + 144,
# 2 = bin NC 192 (one wave per SIMD each)
NUM_SOLVE_KERNELS = 3
KERNEL_BINS = ((1, 0), (3, 2), (4,))
KERNEL_NAMES = ("solve_group_kernel<128, 96>", "solve_group_kernel<160, 144>",
                "solve_group_kernel<192, 0>")

_lib = None


def load(path: str | Path | None = None) -> ctypes.CDLL:
    """Load libcmpc.so (in-tree; $CMPC_LIB names a variant build, e.g. a diagnostic one) and
    declare the prototypes.  Raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is None and os.environ.get("CMPC_LIB"):
        path = os.environ["CMPC_LIB"]
    p = Path(path) if path is not None else LIB
    if not p.exists():
        raise RuntimeError(f"cmpc: HIP library {p} not built (run __graft_entry__.build() or "
                           f"python -m cmpc.build); there is no CPU fallback")
    lib = ctypes.CDLL(str(p))
    vp = ctypes.c_void_p
    lib.cmpc_params_default.argtypes = [ctypes.POINTER(CParams)]
    lib.cmpc_params_default.restype = None
    lib.cmpc_plan_create.argtypes = [ctypes.POINTER(CParams), ctypes.POINTER(vp)]
    lib.cmpc_plan_create.restype = ctypes.c_int
    lib.cmpc_solve.argtypes = [vp, ctypes.c_int64] + [vp] * 10
    lib.cmpc_solve.restype = ctypes.c_int
    if hasattr(lib, "cmpc_solve_warm"):  # absent from A/B builds of older sources
        lib.cmpc_solve_warm.argtypes = [vp, ctypes.c_int64] + [vp] * 13
        lib.cmpc_solve_warm.restype = ctypes.c_int
    if hasattr(lib, "cmpc_solve_ref"):
        lib.cmpc_solve_ref.argtypes = [vp, ctypes.c_int64] + [vp] * 13
        lib.cmpc_solve_ref.restype = ctypes.c_int
    lib.cmpc_build_dynamics.argtypes = [vp, ctypes.c_int64, ctypes.c_float] + [vp] * 8
    lib.cmpc_build_dynamics.restype = ctypes.c_int
    if hasattr(lib, "cmpc_generate_traj"):
        lib.cmpc_generate_traj.argtypes = [vp, ctypes.c_int64, ctypes.c_double] + [vp] * 11
        lib.cmpc_generate_traj.restype = ctypes.c_int
    if hasattr(lib, "cmpc_leg_torque"):
        lib.cmpc_leg_torque.argtypes = ([vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64] +
                                        [vp] * 12 + [ctypes.c_double, vp, vp])
        lib.cmpc_leg_torque.restype = ctypes.c_int
    if hasattr(lib, "cmpc_srb_step"):
        lib.cmpc_srb_step.argtypes = ([vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double] + [vp] * 5 +
                                      [ctypes.c_int64] + [vp] * 5)
        lib.cmpc_srb_step.restype = ctypes.c_int
    lib.cmpc_plan_destroy.argtypes = [vp]
    lib.cmpc_plan_destroy.restype = None
    lib.cmpc_plan_set_timing.argtypes = [vp, ctypes.c_int]
    lib.cmpc_plan_set_timing.restype = ctypes.c_int
    lib.cmpc_plan_timing_read.argtypes = [vp, ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(ctypes.c_int32)]
    lib.cmpc_plan_timing_read.restype = ctypes.c_int
    if hasattr(lib, "cmpc_plan_set_team"):
        lib.cmpc_plan_set_team.argtypes = [vp, ctypes.c_int64]
        lib.cmpc_plan_set_team.restype = ctypes.c_int
        lib.cmpc_plan_team_batch.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
        lib.cmpc_plan_team_batch.restype = ctypes.c_int
    if hasattr(lib, "cmpc_plan_set_heavy_first"):
        lib.cmpc_plan_set_heavy_first.argtypes = [vp, ctypes.c_int64]
        lib.cmpc_plan_set_heavy_first.restype = ctypes.c_int
        lib.cmpc_plan_heavy_first_batch.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
        lib.cmpc_plan_heavy_first_batch.restype = ctypes.c_int
    if hasattr(lib, "cmpc_plan_stats"):
        lib.cmpc_plan_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        lib.cmpc_plan_stats.restype = ctypes.c_int
    if hasattr(lib, "cmpc_plan_solve_kernel"):
        lib.cmpc_plan_solve_kernel.argtypes = [vp, ctypes.c_int64, ctypes.c_int]
        lib.cmpc_plan_solve_kernel.restype = ctypes.c_char_p
    lib.cmpc_last_error.argtypes = []
    lib.cmpc_last_error.restype = ctypes.c_char_p
    lib.cmpc_version.argtypes = []
    lib.cmpc_version.restype = ctypes.c_char_p
    if path is None:
        _lib = lib
    return lib


def last_error(lib=None) -> str:
    lib = lib or load()
    return lib.cmpc_last_error().decode()
