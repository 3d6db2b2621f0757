"""Shared helpers for the parity tests (TEST INFRASTRUCTURE)."""
from __future__ import annotations

import numpy as np

from conftest import GOLDEN


def load_fixture(name):
    z = np.load(GOLDEN / name, allow_pickle=False)
    return {k: z[k] for k in z.files}


def fixture_batch(fx):
    return {k: fx[k] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}


def split_w(w, N=16):
    """w (B, 24N) reference layout -> X (B, N, 12) = x_1..x_N, U (B, N, 12) = u_0..u_{N-1}."""
    B = w.shape[0]
    return w[:, :12 * N].reshape(B, N, 12), w[:, 12 * N:].reshape(B, N, 12)


def rel_err_U(w_gpu, w_ref, N=16):
    _, Ug = split_w(np.asarray(w_gpu, np.float64), N)
    _, Ur = split_w(np.asarray(w_ref, np.float64), N)
    num = np.max(np.abs(Ug - Ur).reshape(len(Ug), -1), axis=1)
    den = np.max(np.abs(Ur).reshape(len(Ur), -1), axis=1)
    return num / np.maximum(den, 1e-12)


def rollout64(batch, U):
    """x_{k+1} = Ad x_k + Bd_k u_k + gd in float64 for a batch: (B, N, 12)."""
    Ad, Bd, gd, x0 = batch["Ad"], batch["Bd"], batch["gd"], batch["x0"]
    B, N = Bd.shape[:2]
    X = np.zeros((B, N, 12))
    x = x0.astype(np.float64)
    for k in range(N):
        x = np.einsum("bij,bj->bi", Ad, x) + np.einsum("bij,bj->bi", Bd[:, k], U[:, k]) + gd
        X[:, k] = x
    return X


def feasibility(batch, U, mu=0.8, fz_min=10.0):
    """Max violation of the reference's bounds/friction rows (centroidal_mpc.py:122-176,
    264-283, 324-359) per instance (absolute, Newtons)."""
    ct = batch["contact"].transpose(0, 2, 1).astype(bool)      # (B, N, 4)
    F = U.reshape(U.shape[0], U.shape[1], 4, 3)
    fx, fy, fz = F[..., 0], F[..., 1], F[..., 2]
    v_sw = np.where(~ct, np.abs(F).max(-1), 0.0)
    v_st = np.where(ct, np.maximum.reduce([fz_min - fz, np.abs(fx) - mu * fz,
                                           np.abs(fy) - mu * fz, np.zeros_like(fz)]), 0.0)
    return np.maximum(v_sw, v_st).reshape(U.shape[0], -1).max(1)


def assert_verified(st, max_unverified=1e-4):
    """A large synthetic batch: every instance solved, status 1 (KKT-verified, within 1e-4 of the
    optimum by the certified bound, include/cmpc.h) except at most a max_unverified fraction at
    status 2 -- a polished point that missed the certified face bound and is returned without
    the 1e-4 guarantee (config 3: 1 of 65,536).  Returns the status-1 mask."""
    st = np.asarray(st)
    assert np.all((st == 1) | (st == 2)), np.unique(st, return_counts=True)
    assert np.sum(st == 2) <= max(1, int(max_unverified * len(st))), np.flatnonzero(st == 2)[:16]
    return st == 1


def input_digest(batch, idx):
    """sha256 of the fp32 boundary inputs of instances `idx` (detects generator drift between
    the fixture's generation and the test)."""
    import hashlib
    h = hashlib.sha256()
    for k in ("Ad", "Bd", "gd", "x0", "xref"):
        h.update(np.ascontiguousarray(batch[k][idx], dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(batch["contact"][idx], dtype=np.uint8).tobytes())
    return h.hexdigest()
