"""Diagnostic: status and max iterations of the hard-case fixture (tests/golden/qp_hard.npz,
each instance replicated 1,100x) under a given build: python tools/hard_iters.py <lib.so>."""
import sys, numpy as np
sys.path.insert(0, 'convex-mpc-unitree-go2_amd'); sys.path.insert(0, 'tests')
import torch
from cmpc import _lib
_lib._lib = _lib.load(sys.argv[1])
from cmpc import Plan, SolverParams, solve_batch
from parity_util import load_fixture, fixture_batch
fx = load_fixture("qp_hard.npz"); reps = 1100
batch = {k: np.repeat(v, reps, axis=0) for k, v in fixture_batch(fx).items()}
w, st, it = solve_batch(batch, plan=Plan(SolverParams(max_batch=65536)))
print(sys.argv[1].split('/')[-1], "status", np.unique(st).tolist(), "iters", [int(it[i*reps:(i+1)*reps].max()) for i in range(4)])
