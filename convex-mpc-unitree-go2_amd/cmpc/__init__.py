"""cmpc -- MI355X-native batched convex-MPC contact-force QP solver.

Drop-in for the CasADi/OSQP solve of ltinphan/convex-mpc-unitree-go2
(convex_mpc/centroidal_mpc.py).  See DESIGN.md.
"""
from .solver import (Plan, SolverParams, CmpcError, solve_batch, to_device_batch,  # noqa: F401
                     leg_state, STATUS_STRINGS)

__version__ = "0.1.0"
