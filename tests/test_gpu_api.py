"""GPU: the drop-in CentroidalMPC API (centroidal_mpc.py) on a trajectory produced by the
reference's own ComTraj.generate_traj (tests/golden/ref_inputs.npz, case 0)."""
import numpy as np
import pytest

from parity_util import load_fixture

pytestmark = pytest.mark.gpu


class Traj:
    """The ComTraj fields CentroidalMPC reads (centroidal_mpc.py:204-269)."""

    def __init__(self, c):
        self.N = int(c["N"])
        self.Ad = c["Ad"]
        self.Bd = c["Bd"]
        self.gd = c["gd"].reshape(-1, 1)
        self.initial_x_vec = c["x0"].reshape(-1, 1)
        self.contact_table = c["contact"]
        self._xref = c["xref"]

    def compute_x_ref_vec(self):
        return self._xref


def _case(i):
    z = load_fixture("ref_inputs.npz")
    return {k[len(f"c{i}_"):]: v for k, v in z.items() if k.startswith(f"c{i}_")}


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_centroidal_mpc_dropin(ci, capsys):
    from centroidal_mpc import CentroidalMPC
    from oracle import mpc_qp, tight_solver
    c = _case(ci)
    traj = Traj(c)
    mpc = CentroidalMPC(None, traj)
    out = capsys.readouterr().out
    assert "A:  448 x 384  | nnz =   5168" in out or traj.N != 16
    sol = mpc.solve_QP(None, traj, verbose=True)
    assert "[QP SOLVER] status: solved" in capsys.readouterr().out
    N = traj.N
    w = sol["x"].full().flatten()                   # test_MPC.py:190
    assert w.shape == (24 * N,)
    X_opt = w[:12 * N].reshape((12, N), order="F")  # test_MPC.py:191-192
    U_opt = w[12 * N:].reshape((12, N), order="F")
    qp = mpc_qp.build_qp(c["Ad"], c["Bd"], c["gd"], c["x0"], c["xref"], c["contact"])
    r = tight_solver.solve(qp)
    Xr, Ur = mpc_qp.unpack_w(r["w"])
    assert np.max(np.abs(U_opt - Ur)) / np.max(np.abs(Ur)) <= 1e-4
    assert mpc.solve_time > 0 and mpc.update_time > 0
    assert mpc.solver.stats()["return_status"] == "solved"
    assert sol["lam_a"].full().shape == (28 * N, 1) and sol["lam_x"].full().shape == (24 * N, 1)
    k = mpc_qp.kkt_residuals(qp, w, sol["lam_x"].full().ravel(), sol["lam_a"].full().ravel())
    assert k["prim"] < 1e-3 and k["stat"] < 1e-3 * (1 + np.max(np.abs(qp["g"])))
    # second tick is warm-started from the first (centroidal_mpc.py:91-95): the same optimum,
    # reached by the direct polish of the warm face set (no ADMM iteration)
    sol2 = mpc.solve_QP(None, traj)
    U2 = sol2["x"].full().flatten()[12 * N:].reshape((12, N), order="F")
    assert np.max(np.abs(U2 - Ur)) / np.max(np.abs(Ur)) <= 1e-4
    assert mpc.solver.stats()["return_status"] == "solved"
    assert mpc.solver.stats()["iter_count"] == 0
