"""Conversion-only stand-in for the ``casadi`` module (TEST INFRASTRUCTURE, fixture generation).

CasADi 3.6.7 is not installed in this image (an ordinary ModuleNotFoundError).
The reference's QP *assembly* -- ``CentroidalMPC.__init__``, ``_compute_bounds``,
``_update_sparse_matrix``, ``_assemble_A_matrix``, ``_create_dynamics_function``,
``_precompute_friction_matrix``, ``_build_sparse_matrix`` (centroidal_mpc.py:41-67, 122-359) --
uses CasADi only to hold matrices and to concatenate / multiply them.  This module provides
exactly that subset, so those functions run UNMODIFIED from /root/reference and their outputs
become golden vectors (tests/golden/make_golden.py ``make_qp_assembly``):

* ``DM``: a float64 matrix with a structural-nonzero mask (CasADi keeps structural zeros:
  ``DM(ndarray)`` is dense, ``DM.eye`` / ``DM.triplet`` / ``DM(Sparsity, data)`` are sparse;
  ``@`` unions the boolean product pattern, ``+`` the union, scalar ``*`` keeps the pattern);
* ``Sparsity(nrow, ncol, colind, row)`` (CSC), ``nnz()``, ``size()``;
* ``vec`` (column-major), ``vertcat``, ``horzcat``, ``repmat``, ``diagcat``, ``inf``;
* ``SX.sym`` / slicing / unary minus / ``diagcat`` and ``Function``: an SX element here is
  ``coef * symbol`` or a structural zero -- the only expressions ``_create_dynamics_function``
  builds (it negates and block-diagonalises the symbolic Ad / Bd_seq);
* ``conic``: returns a handle that records its arguments and cannot solve (OSQP is absent).

Nothing here computes a QP solution; it only reproduces the data the reference hands to the
solver.
"""
from __future__ import annotations

import numpy as np

inf = np.inf


class Sparsity:
    def __init__(self, nrow, ncol, colind=None, row=None, mask=None):
        if mask is None:
            mask = np.zeros((nrow, ncol), dtype=bool)
            colind = np.asarray(colind)
            row = np.asarray(row)
            for j in range(ncol):
                mask[row[colind[j]:colind[j + 1]], j] = True
        self.mask = np.asarray(mask, dtype=bool)

    def nnz(self):
        return int(self.mask.sum())

    def size(self):
        return self.mask.shape

    def size1(self):
        return self.mask.shape[0]

    def size2(self):
        return self.mask.shape[1]

    def csc(self):
        """(colind, row) of the pattern, CasADi's CSC order."""
        cols, rows = np.nonzero(self.mask.T)
        colind = np.concatenate([[0], np.cumsum(np.bincount(cols, minlength=self.mask.shape[1]))])
        return colind, rows


class DM:
    """Dense values + structural mask."""

    def __init__(self, a=None, data=None):
        if isinstance(a, Sparsity):
            v = np.zeros(a.mask.shape)
            d = np.asarray(data, dtype=np.float64).reshape(-1, order="F")
            v.T[a.mask.T] = d          # CSC order = column-major order of the mask
            self.v, self.m = v, a.mask.copy()
            return
        if isinstance(a, DM):
            self.v, self.m = a.v.copy(), a.m.copy()
            return
        arr = np.asarray(0.0 if a is None else a, dtype=np.float64)
        if arr.ndim == 0:
            arr = arr.reshape(1, 1)
        elif arr.ndim == 1:
            arr = arr.reshape(-1, 1)        # CasADi: a 1-D sequence is a column
        self.v = arr.copy()
        self.m = np.ones(arr.shape, dtype=bool)

    @staticmethod
    def _raw(v, m):
        o = DM.__new__(DM)
        o.v, o.m = v, m
        return o

    # -- constructors --
    @staticmethod
    def eye(n):
        return DM._raw(np.eye(n), np.eye(n, dtype=bool))

    @staticmethod
    def zeros(n, m=1):
        return DM._raw(np.zeros((n, m)), np.zeros((n, m), dtype=bool))

    @staticmethod
    def ones(n, m=1):
        return DM._raw(np.ones((n, m)), np.ones((n, m), dtype=bool))

    @staticmethod
    def triplet(rows, cols, vals, nr, nc):
        v = np.zeros((nr, nc))
        m = np.zeros((nr, nc), dtype=bool)
        vals = vals.v.reshape(-1, order="F") if isinstance(vals, DM) else np.asarray(vals, float)
        for r, c, x in zip(rows, cols, vals):
            v[r, c] += x
            m[r, c] = True
        return DM._raw(v, m)

    # -- queries --
    def sparsity(self):
        return Sparsity(*self.m.shape, mask=self.m)

    def size(self):
        return self.v.shape

    def size1(self):
        return self.v.shape[0]

    def size2(self):
        return self.v.shape[1]

    def nnz(self):
        return int(self.m.sum())

    def full(self):
        return self.v.copy()

    def nonzeros(self):
        return list(self.v.T[self.m.T])

    @property
    def shape(self):
        return self.v.shape

    # -- arithmetic --
    def __matmul__(self, o):
        o = _dm(o)
        return DM._raw(self.v @ o.v, (self.m.astype(np.int64) @ o.m.astype(np.int64)) > 0)

    def __rmatmul__(self, o):
        return _dm(o).__matmul__(self)

    def __add__(self, o):
        o = _dm(o)
        return DM._raw(self.v + o.v, self.m | o.m)

    __radd__ = __add__

    def __sub__(self, o):
        o = _dm(o)
        return DM._raw(self.v - o.v, self.m | o.m)

    def __neg__(self):
        return DM._raw(-self.v, self.m.copy())

    def __mul__(self, o):
        if np.isscalar(o):
            return DM._raw(self.v * o, self.m.copy())
        o = _dm(o)
        return DM._raw(self.v * o.v, self.m & o.m)

    __rmul__ = __mul__

    def __getitem__(self, idx):
        return DM._raw(np.atleast_2d(self.v[idx]), np.atleast_2d(self.m[idx]))


def _dm(x):
    return x if isinstance(x, DM) else DM(x)


# ---- concatenation ------------------------------------------------------------------------
def _parts(args):
    return [a if isinstance(a, (DM, SX)) else DM(a) for a in args]


def vertcat(*args):
    p = _parts(args)
    if any(isinstance(a, SX) for a in p):
        return SX._cat(p, axis=0)
    return DM._raw(np.vstack([a.v for a in p]), np.vstack([a.m for a in p]))


def horzcat(*args):
    p = _parts(args)
    if any(isinstance(a, SX) for a in p):
        return SX._cat(p, axis=1)
    return DM._raw(np.hstack([a.v for a in p]), np.hstack([a.m for a in p]))


def repmat(a, n, m=1):
    a = _dm(a)
    return DM._raw(np.tile(a.v, (n, m)), np.tile(a.m, (n, m)))


def vec(a):
    a = _dm(a)
    return DM._raw(a.v.reshape(-1, 1, order="F"), a.m.reshape(-1, 1, order="F"))


def diagcat(*args):
    p = _parts(args)
    if any(isinstance(a, SX) for a in p):
        return SX._diag(p)
    nr = sum(a.v.shape[0] for a in p)
    nc = sum(a.v.shape[1] for a in p)
    v = np.zeros((nr, nc))
    m = np.zeros((nr, nc), dtype=bool)
    r = c = 0
    for a in p:
        h, w = a.v.shape
        v[r:r + h, c:c + w] = a.v
        m[r:r + h, c:c + w] = a.m
        r += h
        c += w
    return DM._raw(v, m)


# ---- symbolic: coef * symbol per element ---------------------------------------------------
class SX:
    _next = 0

    def __init__(self, sid, coef):
        self.sid = sid          # (r, c) symbol index, -1 = structural zero
        self.coef = coef        # (r, c) float

    @staticmethod
    def sym(name, r, c=1):
        n = r * c
        sid = (SX._next + np.arange(n)).reshape((r, c), order="F")   # column-major elements
        SX._next += n
        return SX(sid, np.ones((r, c)))

    @property
    def shape(self):
        return self.sid.shape

    def __getitem__(self, idx):
        return SX(np.atleast_2d(self.sid[idx]), np.atleast_2d(self.coef[idx]))

    def __neg__(self):
        return SX(self.sid.copy(), -self.coef)

    @staticmethod
    def _lift(a):
        if isinstance(a, SX):
            return a
        if np.any(a.m & (a.v != 0)):
            raise NotImplementedError("stand-in SX holds only coef * symbol expressions")
        return SX(np.full(a.v.shape, -1), np.zeros(a.v.shape))

    @staticmethod
    def _cat(parts, axis):
        p = [SX._lift(a) for a in parts]
        f = np.vstack if axis == 0 else np.hstack
        return SX(f([a.sid for a in p]), f([a.coef for a in p]))

    @staticmethod
    def _diag(parts):
        p = [SX._lift(a) for a in parts]
        nr = sum(a.shape[0] for a in p)
        nc = sum(a.shape[1] for a in p)
        sid = np.full((nr, nc), -1)
        coef = np.zeros((nr, nc))
        r = c = 0
        for a in p:
            h, w = a.shape
            sid[r:r + h, c:c + w] = a.sid
            coef[r:r + h, c:c + w] = a.coef
            r += h
            c += w
        return SX(sid, coef)


class Function:
    """Evaluates SX outputs (coef * symbol) at numeric inputs; positional call -> tuple."""

    def __init__(self, name, inputs, outputs, *a, **k):
        self.name = name
        self.inputs = inputs
        self.outputs = outputs

    def __call__(self, *args):
        val = {}
        for sx, a in zip(self.inputs, args):
            a = _dm(a)
            if a.v.shape != sx.shape:
                raise ValueError(f"{self.name}: input shape {a.v.shape} != {sx.shape}")
            for s, x in zip(sx.sid.reshape(-1, order="F"), a.v.reshape(-1, order="F")):
                val[int(s)] = x
        lut = np.zeros(max(val) + 1)
        for s, x in val.items():
            lut[s] = x
        outs = []
        for o in self.outputs:
            m = o.sid >= 0
            v = np.where(m, o.coef * lut[np.where(m, o.sid, 0)], 0.0)
            outs.append(DM._raw(v, m))
        return tuple(outs) if len(outs) > 1 else outs[0]


class _Conic:
    """ca.conic handle: records the problem structure; solving needs OSQP, which is absent."""

    def __init__(self, name, solver, qp, opts):
        self.name, self.solver, self.qp, self.opts = name, solver, qp, opts

    def __call__(self, **kw):
        raise RuntimeError("casadi stand-in: no QP solver (OSQP is not installed)")

    def stats(self):
        return {}


def conic(name, solver, qp, opts=None):
    return _Conic(name, solver, qp, opts or {})
