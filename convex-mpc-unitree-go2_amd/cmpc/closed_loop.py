"""Batched closed loop on the device: many robots, one MPC tick per call, everything resident.

The reference's loop (test_MPC.py:160-236) runs per robot on the CPU: every STEPS_PER_MPC leg
ticks it calls ``traj.generate_traj`` and ``mpc.solve_QP`` (warm-started) and holds U[:, 0]
until the next MPC tick; MuJoCo integrates the robot.  Here one call of :meth:`ClosedLoop.tick`
does that for B robots with no host round trip:

  cmpc_generate_traj -> cmpc_build_dynamics -> cmpc_solve_warm -> cmpc_srb_step (nsub substeps)

MuJoCo and the Go2 model are absent from this image, so the plant is ``cmpc_srb_step``'s
single-rigid-body stand-in (include/cmpc.h) and the robot quantities Pinocchio would supply are
the synthetic ones of :mod:`cmpc.synth` (mass, body inertia, hip offsets).  :meth:`capture`
records one tick as a HIP graph (``torch.cuda.CUDAGraph``) so that a tick is one graph launch.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import synth
from .solver import Plan, SolverParams, _check


def rot_zyx(rpy: torch.Tensor) -> torch.Tensor:
    """(B,3) roll, pitch, yaw -> (B,3,3) R_z R_y R_x (the base rotation whose ZYX angles are the
    MPC state's rpy, go2_robot_data.py:211-216)."""
    r, p, y = rpy.unbind(-1)
    cr, sr, cp, sp, cy, sy = r.cos(), r.sin(), p.cos(), p.sin(), y.cos(), y.sin()
    return torch.stack([cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr,
                        sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr,
                        -sp, cp * sr, cp * cr], -1).reshape(-1, 3, 3)


class ClosedLoop:
    """B robots walking under batched MPC (test_MPC.py's loop shape, MPC_DT = gait period / N)."""

    def __init__(self, B: int, plan: Optional[Plan] = None, gait_hz: float = synth.GAIT_HZ,
                 duty: float = synth.GAIT_DUTY, offsets=synth.TROT_OFFSETS, nsub: int = 20,
                 seed: int = 0, device="cuda", shift_warm: bool = True):
        self.plan = plan or Plan(SolverParams(max_batch=B))
        self.B, self.N = B, self.plan.params.N
        dev = torch.device(device)
        self.dev = dev
        self.period = 1.0 / gait_hz
        self.dt = self.period / self.N                    # test_MPC.py:67-68
        self.nsub = nsub                                  # leg ticks per MPC tick (:69)
        f32, f64 = torch.float32, torch.float64
        rng = np.random.default_rng(seed)
        yaw0 = rng.uniform(-np.pi, np.pi, B)
        x = np.zeros((B, 12))
        x[:, 0:2] = rng.uniform(-1, 1, (B, 2))
        x[:, 2] = synth.Z_DES
        x[:, 5] = yaw0
        self.x = torch.as_tensor(x, dtype=f32, device=dev).contiguous()
        self.pos_des = self.x[:, 0:3].to(f64).clone()     # ComTraj.__init__ (com_trajectory.py:12-13)
        self.t = torch.zeros(B, dtype=f64, device=dev)
        self.gait = torch.tensor([self.period, duty, *offsets], dtype=f64,
                                 device=dev).repeat(B, 1).contiguous()
        self.hip = torch.as_tensor(synth.HIP_OFFSETS, dtype=f32, device=dev).contiguous()
        self.mass = torch.full((B,), synth.MASS, dtype=f32, device=dev)
        self.I_body = torch.as_tensor(synth.INERTIA_BODY, dtype=f32, device=dev).repeat(B, 1, 1).contiguous()
        c, s = np.cos(yaw0), np.sin(yaw0)
        hipw = np.stack([np.stack([x[:, 0] + c * hx - s * hy, x[:, 1] + s * hx + c * hy,
                                   np.zeros(B)], -1) for hx, hy in synth.HIP_XY], 1)
        self.feet = torch.as_tensor(hipw, dtype=f32, device=dev).contiguous()
        self.contact = torch.full((B,), 0xF, dtype=torch.uint8, device=dev)
        N = self.N
        self.cmd = torch.zeros((B, 4), dtype=f32, device=dev)
        self.cmd[:, 2] = synth.Z_DES
        self.xref = torch.empty((B, N, 12), dtype=f32, device=dev)
        self.ct = torch.empty((B, 4, N), dtype=torch.uint8, device=dev)
        self.rf = torch.empty((B, N, 4, 3), dtype=f32, device=dev)
        self.Ad = torch.empty((B, 12, 12), dtype=f32, device=dev)
        self.Bd = torch.empty((B, N, 12, 12), dtype=f32, device=dev)
        self.gd = torch.empty((B, 12), dtype=f32, device=dev)
        self.w = torch.zeros((B, 24 * N), dtype=f32, device=dev)
        self.y = torch.zeros((B, 12 * N), dtype=f32, device=dev)
        self.status = torch.empty((B,), dtype=torch.int32, device=dev)
        self.iters = torch.empty((B,), dtype=torch.int32, device=dev)
        self.lever = torch.empty((B, 4, 3), dtype=f32, device=dev)
        self.I_world = torch.empty((B, 3, 3), dtype=f32, device=dev)
        self.w_init = torch.zeros_like(self.w)
        self.y_init = torch.zeros_like(self.y)
        self.shift_warm = shift_warm
        self.warm = False
        self.graph = None

    def set_command(self, cmd):
        """(B,4) [vx_body, vy_body, z_des, yaw_rate] (test_MPC.py get_body_cmd)."""
        self.cmd.copy_(torch.as_tensor(cmd, dtype=torch.float32, device=self.dev))

    def _tick(self, stream, warm: bool):
        p, N, B = self.plan, self.N, self.B
        # what generate_traj reads off the robot: levers COM -> foot, I_com in the world frame
        torch.sub(self.feet, self.x[:, None, 0:3], out=self.lever)
        R = rot_zyx(self.x[:, 3:6])
        # R I_body R' as broadcast products + size-3 sums: batched 3x3 GEMMs go to the BLAS
        # library, two launches of ~0.57 ms each at 65,536 robots (rocprofv3, tools/loop_graph.py)
        RI = (R[:, :, :, None] * self.I_body[:, None, :, :]).sum(2)
        torch.sum(RI[:, :, None, :] * R[:, None, :, :], 3, out=self.I_world)
        p.generate_traj(self.x, self.pos_des, self.cmd, self.t, self.gait, self.lever, self.hip,
                        self.dt, out=(self.xref, self.ct, self.rf), stream=stream)
        p.build_dynamics(self.mass, self.I_world, self.rf, self.xref, self.dt,
                         out=(self.Ad, self.Bd, self.gd), stream=stream)
        if warm and self.shift_warm:
            # the previous tick's plan, moved one MPC step forward (its step k+1 is this tick's k;
            # the last step repeats): the contact schedule shifts the same way, so the warm face
            # set lines up with this tick's QP
            U, Ui = self.w[:, 12 * N:].view(B, N, 12), self.w_init[:, 12 * N:].view(B, N, 12)
            Ui[:, :-1].copy_(U[:, 1:]); Ui[:, -1].copy_(U[:, -1])
            Y, Yi = self.y.view(B, N, 12), self.y_init.view(B, N, 12)
            Yi[:, :-1].copy_(Y[:, 1:]); Yi[:, -1].copy_(Y[:, -1])
            kw = dict(w_init=self.w_init, y_init=self.y_init)
        else:
            kw = dict(w_init=self.w, y_init=self.y) if warm else {}
        p.solve(self.Ad, self.Bd, self.gd, self.x, self.xref, self.ct,
                out=(self.w, self.status, self.iters), stream=stream, y_out=self.y, **kw)
        sp = ctypes.c_void_p(stream.cuda_stream)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        force = self.w[:, 12 * N:]                        # U[:, 0] rows (test_MPC.py:196)
        with torch.cuda.device(self.dev):
            rc = p.lib.cmpc_srb_step(p._h, ctypes.c_int64(B), ctypes.c_int(self.nsub),
                                     ctypes.c_double(self.dt / self.nsub), P(self.t), P(self.gait),
                                     P(self.mass), P(self.I_body), P(force),
                                     ctypes.c_int64(self.w.stride(0)), P(self.hip), P(self.x),
                                     P(self.feet), P(self.contact), sp)
        _check(p.lib, rc, "cmpc_srb_step")
        self.t.add_(self.dt)

    def tick(self):
        """One MPC tick for every robot (graph replay once :meth:`capture` has run)."""
        if self.graph is not None:
            self.graph.replay()
            return
        self._tick(torch.cuda.current_stream(self.dev), self.warm)
        self.warm = True

    def capture(self):
        """Record one warm tick as a HIP graph (after at least one eager tick)."""
        if not self.warm:
            self.tick()
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._tick(s, True)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.graph = g
        # capture recorded the work without running it: nothing to undo
