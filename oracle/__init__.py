"""CPU oracle for the batched convex-MPC QP path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import, call, link or execute anything in this directory, and only as the checker (or the
timed CPU baseline), never as the thing measured or shipped.  See DESIGN.md "Oracle".
"""
