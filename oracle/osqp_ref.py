"""CPU ORACLE / BASELINE (test infrastructure only) -- Python binding of oracle/osqp_ref.cpp.

``osqp_ref.cpp`` restates the reference's per-tick QP solve (CasADi 3.6.7 conic plugin
'osqp' with the reference OPTS, centroidal_mpc.py:20-36, :98, :213) in float64.  Used by
``bench.py`` as the ``cpu_baseline`` ("kind": "port") and by tests to report the distance of
the HIP solution to an OSQP-like output (informational; the parity target is the
KKT-certified optimum of oracle/tight_solver.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libosqp_ref.so"


class Settings(ctypes.Structure):
    _fields_ = [("Q", ctypes.c_double * 12), ("R", ctypes.c_double * 12),
                ("mu", ctypes.c_double), ("fz_min", ctypes.c_double),
                ("rho", ctypes.c_double), ("sigma", ctypes.c_double),
                ("alpha", ctypes.c_double), ("eps_abs", ctypes.c_double),
                ("eps_rel", ctypes.c_double), ("adaptive_rho_tolerance", ctypes.c_double),
                ("max_iter", ctypes.c_int), ("check_termination", ctypes.c_int),
                ("adaptive_rho_interval", ctypes.c_int), ("scaling", ctypes.c_int),
                ("scaled_termination", ctypes.c_int)]


def build(force: bool = False) -> Path:
    src = HERE / "osqp_ref.cpp"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = ctypes.CDLL(str(LIB))
        _lib.osqp_ref_default.argtypes = [ctypes.POINTER(Settings)]
        _lib.osqp_ref_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6 + \
            [ctypes.POINTER(Settings)] + [ctypes.c_void_p] * 5 + [ctypes.c_int]
        _lib.osqp_ref_solve_batch.restype = ctypes.c_int
    return _lib


def default_settings() -> Settings:
    s = Settings()
    lib().osqp_ref_default(ctypes.byref(s))
    return s


def solve_batch(batch: dict, threads: int = 1, settings: Settings | None = None):
    """OSQP-restatement solve of a numpy batch (cmpc.synth layout).  Returns dict with
    w (B, 24N), lam_x (B, 24N), lam_a (B, 28N), status, iters."""
    s = settings or default_settings()
    B, N = batch["Bd"].shape[:2]
    arr = {k: np.ascontiguousarray(batch[k], dtype=np.float64) for k in ("Ad", "Bd", "gd", "x0", "xref")}
    ct = np.ascontiguousarray(batch["contact"], dtype=np.uint8)
    w = np.zeros((B, 24 * N))
    lx = np.zeros((B, 24 * N))
    la = np.zeros((B, 28 * N))
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib().osqp_ref_solve_batch(B, N, p(arr["Ad"]), p(arr["Bd"]), p(arr["gd"]), p(arr["x0"]),
                               p(arr["xref"]), p(ct), ctypes.byref(s), p(w), p(lx), p(la),
                               p(st), p(it), threads)
    return dict(w=w, lam_x=lx, lam_a=la, status=st, iters=it)


def time_baseline(batch: dict, seconds: float = 15.0):
    """Time the OSQP restatement on the host: single-thread latency on a small sample and
    all-core throughput on a bounded sample of the same workload (~``seconds`` total)."""
    cores = len(os.sched_getaffinity(0))
    cores = max(1, min(cores, 16))      # the GPU box grants 16 host cores per GPU
    B = batch["Bd"].shape[0]
    sub = lambda n: {k: v[:n] for k, v in batch.items() if isinstance(v, np.ndarray)}  # noqa: E731
    n1 = min(B, 16)
    t0 = time.perf_counter()
    solve_batch(sub(n1), threads=1)
    t1 = time.perf_counter()
    per1 = (t1 - t0) / n1
    n_all = int(max(cores, min(B, (seconds * 0.7) / per1 * cores)))
    n_all = min(n_all, B)
    t0 = time.perf_counter()
    r = solve_batch(sub(n_all), threads=cores)
    t1 = time.perf_counter()
    return {"value": n_all / (t1 - t0), "unit": "solves/s", "cores": cores, "kind": "port",
            "sample": f"{n_all} instances of the bench workload, oracle/osqp_ref.cpp (OSQP-0.6 "
                      f"algorithm restated, reference OPTS, cold start, float64), OpenMP x{cores}",
            "single_thread_ms": per1 * 1e3,
            "osqp_solved_frac": float(np.mean(r["status"] == 1)),
            "osqp_iters_mean": float(np.mean(r["iters"])),
            "_w": r["w"]}   # the sample's solutions (instances 0 .. n-1), not printed


def tight_settings() -> Settings:
    """The same restatement run to eps 1e-10: it converges to the KKT-certified optimum
    (tests/test_osqp_port.py), so it measures how far the reference OPTS stop from it."""
    s = default_settings()
    s.eps_abs = s.eps_rel = 1e-10
    s.max_iter = 400000
    return s
