#!/usr/bin/env python3
"""bench.py -- batched convex-MPC QP solves/sec on MI355X (BASELINE.json metric).

One *step* = one cmpc_solve over a resident batch of synthetic Go2 QP instances
(default workload: config 1 distribution -- trot 3 Hz / duty 0.6 fixed
contact schedule, seed 1 -- at ``--batch`` instances per GPU).  Instances are independent, so
ranks shard them with no data-path collective (weak scaling: every rank solves its own
``--batch`` instances, generated rank-locally from seed + rank); only the barrier and the
max-over-ranks timing reduction use the process group.

    python bench.py [--gpus N --steps K --warmup W --config 1|2|3 --batch B]

Rank 0 prints one JSON line.  ``roofline`` prices the dominant solve kernel (the free-variable
bin that holds most instances) against HBM: algorithmic bytes = 12,264 B per solve (inputs
10,720 + outputs 1,544) x solves in that launch / its average HIP-event duration.
``cpu_baseline`` times the oracle's C restatement of the reference's OSQP path
(oracle/osqp_ref.c, float64, the reference's OPTS) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))

BYTES_IN = 576 + 9216 + 48 + 48 + 768 + 64      # Ad, Bd, gd, x0, xref, contact (N=16, fp32/u8)
BYTES_OUT = 1536 + 4 + 4                         # w, status, iters
BYTES_PER_SOLVE = BYTES_IN + BYTES_OUT           # 12,264
HBM_PEAK_GBS = 8000.0                            # MI355X_MICROARCH.md: 8.0 TB/s spec
F32_MATRIX_PEAK_TFS = 157.3                      # MI355X_MICROARCH.md: dense f32 MFMA peak
POLISH_REFINE = 4                                # SolverParams.polish_refine (default)


def algorithmic_flops(contact, iters, N=16):
    """Algorithmic FP32 work per instance of the path's algorithm (DESIGN.md "Roofline"):
    one ADMM and one polish factorisation at the instance's free-force count n (condensation
    sum_t 12 m_t^2 + 288 m_{t-1} with m_t = free forces of steps <= t, sweep inverse n^3),
    `iters` ADMM iterations and POLISH_REFINE refinements of symv (2 n^2) + gradient
    (576 N + 48 n).  Counts only the accepted path (no rho refactors, repairs or padding)."""
    st = (contact != 0).reshape(contact.shape[0], 4, -1)           # (B, 4, N)
    per_step = 3 * st.sum(1).astype(np.float64)                     # free forces per step
    m = np.cumsum(per_step, axis=1)                                 # m_t
    n = m[:, -1]
    m_prev = np.concatenate([np.zeros((m.shape[0], 1)), m[:, :-1]], axis=1)
    cond = (12.0 * m ** 2 + 288.0 * m_prev).sum(1)
    inv = n ** 3
    symv = 2.0 * n ** 2
    grad = 576.0 * N + 48.0 * n
    it = iters.astype(np.float64)
    return 2.0 * (cond + inv) + it * (symv + grad) + POLISH_REFINE * symv + (POLISH_REFINE + 1) * grad


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=1, choices=(1, 2, 3))
    ap.add_argument("--batch", type=int, default=65536, help="instances per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-baseline sample (0 = skip)")
    ap.add_argument("--traffic-json", type=str, default=str(REPO / "profiles" / "hbm_traffic.json"),
                    help="PMC-derived HBM bytes per launch of the dominant kernel (profiles/)")
    ap.add_argument("--latency-batch", type=int, default=256)
    ap.add_argument("--dynamics-steps", type=int, default=5,
                    help="timed steps of the on-device dynamics build (+ fused build+solve); 0 = skip")
    ap.add_argument("--warm-steps", type=int, default=5,
                    help="timed steps of the warm-started next-tick scenario (+ its cold twin); 0 = skip")
    ap.add_argument("--tick-steps", type=int, default=5,
                    help="timed steps of the all-on-device MPC tick (generate_traj -> "
                         "build_dynamics -> solve); 0 = skip")
    ap.add_argument("--leg-steps", type=int, default=5,
                    help="timed steps of the on-device leg controller (cmpc_leg_torque); 0 = skip")
    ap.add_argument("--loop-steps", type=int, default=24,
                    help="timed closed-loop MPC ticks (config 4 shape, SRB plant); 0 = skip")
    ap.add_argument("--api-ticks", type=int, default=20,
                    help="config 0: ticks of one robot through the CentroidalMPC drop-in; 0 = skip")
    ap.add_argument("--seed-offset", type=int, default=0,
                    help="added to the workload seed (experiments: average over batches)")
    ap.add_argument("--param", action="append", default=[],
                    help="SolverParams override key=value (experiments)")
    ap.add_argument("--lib", type=str, default=None,
                    help="alternative build of libcmpc.so (A/B experiments)")
    return ap.parse_args()


def bins_of(contact):
    nf = 3 * (contact != 0).reshape(contact.shape[0], -1).sum(1)
    caps = np.array([96, 128, 160, 192])
    return np.searchsorted(caps, nf)   # first cap >= nf


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    if args.lib:
        from cmpc import _lib
        _lib._lib = _lib.load(args.lib)
    from cmpc import Plan, SolverParams, to_device_batch, synth

    B = args.batch
    cfg = args.config
    if cfg == 3:
        batch = synth.make_config(3, B=B)
    else:
        batch = synth.make_batch(B, seed=synth.CONFIGS[cfg]["seed"] + 1000 * rank + args.seed_offset,
                                 mixed=synth.CONFIGS[cfg]["mixed"])
    bins = bins_of(batch["contact"])
    d = to_device_batch(batch, dev)
    over = {}
    for kv in args.param:
        k, v = kv.split("=")
        over[k] = type(getattr(SolverParams, k))(float(v) if "." in v or "e" in v else int(v))
    plan = Plan(SolverParams(max_batch=B, **over), device=dev)
    w = torch.empty((B, 24 * 16), dtype=torch.float32, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                   out=(w, st, it), stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    plan.timing_read()
    plan.set_timing(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    plan.set_timing(False)
    ms_bins, calls = plan.timing_read()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    status = st.cpu().numpy()
    iters = it.cpu().numpy()
    solved_frac = float(np.mean(status == 1))
    total = B * world * args.steps
    value = total / elapsed

    # dominant kernel: the bin with the most kernel time
    q = int(np.argmax(ms_bins))
    n_in_bin = int(np.sum(bins == q))
    avg_ms = ms_bins[q] / max(calls[q], 1)
    achieved_gbs = BYTES_PER_SOLVE * n_in_bin / (avg_ms * 1e-3) / 1e9
    flops = algorithmic_flops(batch["contact"], iters)
    fl_bin = float(flops[bins == q].sum())
    achieved_tfs = fl_bin / (avg_ms * 1e-3) / 1e12
    traffic = None
    if args.traffic_json and Path(args.traffic_json).exists():
        tj = json.loads(Path(args.traffic_json).read_text())
        traffic = tj.get("hbm_bytes_per_launch")

    # latency of one small batch (configs[1]: B=256) on the same plan (0: skip, e.g. under a
    # profiler so that every traced launch is a full-batch step)
    lb = min(args.latency_batch, B)
    lat_ms = None
    sl = {k: v[:lb] for k, v in d.items()}
    if lb > 0:
        for _ in range(3):
            plan.solve(sl["Ad"], sl["Bd"], sl["gd"], sl["x0"], sl["xref"], sl["contact"])
        torch.cuda.synchronize(dev)
        tl0 = time.perf_counter()
        for _ in range(10):
            plan.solve(sl["Ad"], sl["Bd"], sl["gd"], sl["x0"], sl["xref"], sl["contact"])
        torch.cuda.synchronize(dev)
        lat_ms = (time.perf_counter() - tl0) / 10 * 1e3

    # the discrete dynamics built on the device (cmpc_build_dynamics) --
    # its own HBM roofline, and the fused per-tick throughput build + solve
    dyn = None
    if args.dynamics_steps > 0:
        N = 16
        dm = {k: torch.as_tensor(batch[k], dtype=torch.float32).contiguous().to(dev)
              for k in ("m", "I_world", "r_legs")}
        dt = float(batch["dt"])
        outs = (torch.empty_like(d["Ad"]), torch.empty_like(d["Bd"]), torch.empty_like(d["gd"]))
        for _ in range(2):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.dynamics_steps):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        dyn_ms = e0.elapsed_time(e1) / args.dynamics_steps
        dyn_bytes = B * (4 + 36 + N * 48 + N * 48 + 576 + N * 576 + 48)
        t0f = time.perf_counter()
        for _ in range(args.dynamics_steps):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
            plan.solve(outs[0], outs[1], outs[2], d["x0"], d["xref"], d["contact"],
                       out=(w, st, it), stream=stream)
        torch.cuda.synchronize(dev)
        fused = B * args.dynamics_steps / (time.perf_counter() - t0f)
        gbs = dyn_bytes / (dyn_ms * 1e-3) / 1e9
        dyn = {"kernel": "dynamics_kernel", "ms_per_step": dyn_ms, "robots_per_s": B / (dyn_ms * 1e-3),
               "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": gbs / HBM_PEAK_GBS, "bytes_per_robot": dyn_bytes // B},
               "fused_build_and_solve_per_s": fused}

    # warm start (centroidal_mpc.py:91-95).  Next-tick proxy: the state
    # moves (x0 + noise), reference and gait stay; every warm step starts from the previous
    # tick's (w, y).  Cold and warm solves of the same next-tick batch, same timing method.
    warm = None
    if args.warm_steps > 0:
        y0 = torch.empty((B, 12 * 16), dtype=torch.float32, device=dev)
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                   out=(w, st, it), stream=stream, y_out=y0)
        w0 = w.clone()
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        sc = torch.tensor([2e-3] * 6 + [2e-2] * 6, device=dev)
        d2 = dict(d)
        d2["x0"] = (d["x0"] + torch.randn(d["x0"].shape, generator=g, device=dev) * sc).contiguous()
        y1 = torch.empty_like(y0)

        def timed(warm_on):
            for _ in range(2):
                plan.solve(d2["Ad"], d2["Bd"], d2["gd"], d2["x0"], d2["xref"], d2["contact"],
                           out=(w, st, it), stream=stream,
                           **(dict(w_init=w0, y_init=y0, y_out=y1) if warm_on else {}))
            torch.cuda.synchronize(dev)
            ta = time.perf_counter()
            for _ in range(args.warm_steps):
                plan.solve(d2["Ad"], d2["Bd"], d2["gd"], d2["x0"], d2["xref"], d2["contact"],
                           out=(w, st, it), stream=stream,
                           **(dict(w_init=w0, y_init=y0, y_out=y1) if warm_on else {}))
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - ta
            itn = it.cpu().numpy()
            return (B * args.warm_steps / el, float(itn.mean()), (st == 1).float().mean().item(),
                    int(itn.max()), float(np.percentile(itn, 99.9)))
        cold_rate, cold_it, cold_ok, cold_max, cold_p = timed(False)
        warm_rate, warm_it, warm_ok, warm_max, warm_p = timed(True)
        warm = {"scenario": "next tick: x0 + N(0, 2e-3 pos/rpy, 2e-2 vel/omega); warm from the "
                            "previous tick's (w, y_out), cmpc_solve_warm",
                "solves_per_s_warm": warm_rate, "solves_per_s_cold": cold_rate,
                "speedup": warm_rate / cold_rate, "iters_mean_warm": warm_it,
                "iters_mean_cold": cold_it, "solved_frac_warm": warm_ok,
                "solved_frac_cold": cold_ok, "iters_max_warm": warm_max,
                "iters_max_cold": cold_max, "iters_p999_warm": warm_p, "iters_p999_cold": cold_p}

    # the whole tick on the device -- reference trajectory, contact table
    # and foot levers (cmpc_generate_traj, com_trajectory.py:27-207) -> discrete dynamics -> solve.
    # Inputs are what ComTraj.generate_traj reads from the robot (state, command, time, gait,
    # current levers); the traj kernel gets its own HBM roofline.
    tick = None
    if args.tick_steps > 0:
        tk = synth.make_tick_inputs(B, seed=synth.CONFIGS[min(cfg, 2)]["seed"] + 500 + 1000 * rank,
                                    mixed=cfg != 1)
        f32, f64 = torch.float32, torch.float64
        td = {k: torch.as_tensor(tk[k], dtype=f64 if k in ("pos_des", "t_now", "gait") else f32)
              .contiguous().to(dev) for k in ("x0", "pos_des", "cmd", "t_now", "gait", "foot_lever",
                                              "hip", "m", "I_world")}
        dtt = float(tk["dt"])
        pd0 = td["pos_des"].clone()
        N = 16
        touts = (torch.empty((B, N, 12), dtype=f32, device=dev),
                 torch.empty((B, 4, N), dtype=torch.uint8, device=dev),
                 torch.empty((B, N, 4, 3), dtype=f32, device=dev))
        douts = (torch.empty_like(d["Ad"]), torch.empty_like(d["Bd"]), torch.empty_like(d["gd"]))

        def gen():
            plan.generate_traj(td["x0"], td["pos_des"], td["cmd"], td["t_now"], td["gait"],
                               td["foot_lever"], td["hip"], dtt, out=touts, stream=stream)

        def full_tick():
            gen()
            plan.build_dynamics(td["m"], td["I_world"], touts[2], touts[0], dtt, out=douts,
                                stream=stream)
            plan.solve(douts[0], douts[1], douts[2], td["x0"], touts[0], touts[1],
                       out=(w, st, it), stream=stream)
        for _ in range(2):
            full_tick()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.tick_steps):
            gen()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        tr_ms = e0.elapsed_time(e1) / args.tick_steps
        tr_bytes = 48 + 24 + 16 + 8 + 48 + 48 + N * 48 + 4 * N + N * 48 + 24   # in + out per robot
        t0t = time.perf_counter()
        for _ in range(args.tick_steps):
            full_tick()
        torch.cuda.synchronize(dev)
        tick_rate = B * args.tick_steps / (time.perf_counter() - t0t)
        td["pos_des"].copy_(pd0)
        tick_it = it.cpu().numpy()
        gbs_t = tr_bytes * B / (tr_ms * 1e-3) / 1e9
        tick = {"kernel": "traj_group_kernel", "ms_per_step": tr_ms,
                "roofline": {"bound": "hbm", "achieved": gbs_t, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": gbs_t / HBM_PEAK_GBS, "bytes_per_robot": tr_bytes},
                "full_tick_per_s": tick_rate,
                "full_tick": "generate_traj + build_dynamics + cold solve, all on the device",
                "solved_frac": float((st == 1).float().mean().item()),
                "iters_mean": float(tick_it.mean())}

    # the consumer of U[:, 0] -- the 1 kHz leg controller
    # (leg_controller.py:43-112) for every robot of the batch, on the device, with synthetic
    # Pinocchio quantities (random SPD M) and the solver's own forces.  HBM-bound.
    leg = None
    if args.leg_steps > 0:
        from cmpc import leg_state
        gl = torch.Generator(device=dev).manual_seed(77 + rank)
        f64 = torch.float64
        rn = lambda *sh, s=1.0: torch.randn(sh, generator=gl, device=dev, dtype=f64) * s  # noqa: E731
        Am = rn(B, 18, 18)
        Ml = Am @ Am.transpose(1, 2) / 18 + 0.3 * torch.eye(18, device=dev, dtype=f64)
        del Am
        li = dict(J_foot=rn(B, 4, 3, 3, s=0.2), J_full=rn(B, 4, 3, 18, s=0.2), M=Ml,
                  C=rn(B, 18, 18, s=0.1), g=rn(B, 18, s=3.0), dq=rn(B, 18), Jdot_dq=rn(B, 4, 3, s=0.3),
                  foot_pos=rn(B, 4, 3, s=0.3), foot_vel=rn(B, 4, 3, s=0.3), body=rn(B, 16, s=0.5),
                  hip=rn(4, 3, s=0.2))
        tl = torch.rand(B, generator=gl, device=dev, dtype=f64) * 5
        gait_l = torch.tensor([1 / 3.0, 0.6, 0.5, 0.0, 0.0, 0.5], device=dev, dtype=f64).repeat(B, 1)
        stl = leg_state(B, dev)
        taul = torch.empty((B, 12), dtype=f64, device=dev)

        def leg_step():
            plan.leg_torque(tl, gait_l, w[:, 192:], li["J_foot"], li["J_full"], li["M"], li["C"],
                            li["g"], li["dq"], li["Jdot_dq"], li["foot_pos"], li["foot_vel"],
                            li["body"], li["hip"], stl, out=taul, stream=stream)
        for _ in range(2):
            leg_step()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.leg_steps):
            tl.add_(0.001)
            leg_step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        leg_ms = e0.elapsed_time(e1) / args.leg_steps
        # bytes the controller reads / writes per robot (fp64; C: the 12 leg-joint rows)
        leg_bytes = (8 + 48 + 48 + 288 + 1728 + 2592 + 1728 + 96 + 144 + 96 * 3 + 128 + 256
                     + 96 + 256)
        gbs_l = leg_bytes * B / (leg_ms * 1e-3) / 1e9
        leg = {"kernel": "leg_kernel", "ms_per_step": leg_ms, "robots_per_s": B / (leg_ms * 1e-3),
               "roofline": {"bound": "hbm", "achieved": gbs_l, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": gbs_l / HBM_PEAK_GBS, "bytes_per_robot": leg_bytes},
               "note": "includes the small add_ on t per step; trot gait, 2 legs swing most ticks"}
        del li, Ml

    # BASELINE config 4 shape: robots in closed loop, every MPC tick on the device
    # (generate_traj -> build_dynamics -> warm solve -> SRB plant for 20 leg ticks), recorded once
    # as a HIP graph and replayed.  MuJoCo is absent: the plant is cmpc_srb_step's stand-in.
    loop = None
    if args.loop_steps > 0:
        from cmpc.closed_loop import ClosedLoop
        loop = {"plant": "cmpc_srb_step single-rigid-body stand-in (MuJoCo absent)",
                "mpc_dt_s": 1 / 48}
        for nb in (1024, B):
            cl = ClosedLoop(nb, plan=plan, seed=rank)
            rg = np.random.default_rng(100 + rank)
            cl.set_command(np.stack([rg.uniform(-0.5, 0.5, nb), rg.uniform(-0.2, 0.2, nb),
                                     np.full(nb, 0.27), rg.uniform(-1, 1, nb)], 1))
            for _ in range(4):
                cl.tick()
            torch.cuda.synchronize(dev)
            te = time.perf_counter()
            for _ in range(args.loop_steps):
                cl.tick()
            torch.cuda.synchronize(dev)
            eager = nb * args.loop_steps / (time.perf_counter() - te)
            cl.capture()
            cl.tick()
            torch.cuda.synchronize(dev)
            tg = time.perf_counter()
            for _ in range(args.loop_steps):
                cl.tick()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - tg
            loop[f"robots_{nb}"] = {"robot_ticks_per_s_graph": nb * args.loop_steps / el,
                                    "ms_per_tick_graph": el / args.loop_steps * 1e3,
                                    "robot_ticks_per_s_eager": eager,
                                    "solved_frac": float((cl.status == 1).float().mean().item()),
                                    "iters_mean": float(cl.iters.float().mean().item()),
                                    "com_z_min": float(cl.x[:, 2].min().item())}
            del cl

    # BASELINE config 0: one robot through the reference's own API (CentroidalMPC.solve_QP, the
    # drop-in of centroidal_mpc.py), warm-started every tick as the reference does; the reference
    # budget per MPC tick is MPC_DT = 20.8 ms (test_MPC.py:67-68).
    api = None
    if args.api_ticks > 0 and rank == 0:
        import types
        sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))
        from centroidal_mpc import CentroidalMPC
        one = synth.make_batch(1, seed=0)
        traj = types.SimpleNamespace(
            N=16, Ad=one["Ad"][0], Bd=one["Bd"][0], gd=one["gd"][0].reshape(12, 1),
            initial_x_vec=one["x0"][0].reshape(12, 1), contact_table=one["contact"][0].astype(np.int32),
            compute_x_ref_vec=lambda: one["xref"][0].T.copy())
        import contextlib
        with contextlib.redirect_stdout(sys.stderr):  # the reference's init print (:225-230)
            mpc = CentroidalMPC(None, traj)
        st_ms, up_ms, wall = [], [], []
        for k in range(args.api_ticks + 2):
            ta = time.perf_counter()
            sol = mpc.solve_QP(None, traj, False)
            _ = sol["x"].full()
            if k >= 2:
                wall.append((time.perf_counter() - ta) * 1e3)
                st_ms.append(mpc.solve_time)
                up_ms.append(mpc.update_time)
        api = {"path": "CentroidalMPC(go2, traj).solve_QP -> sol['x'].full(), 1 robot, warm",
               "solve_time_ms": float(np.median(st_ms)), "update_time_ms": float(np.median(up_ms)),
               "wall_ms_per_tick": float(np.median(wall)), "mpc_dt_budget_ms": 1e3 / 48,
               "return_status": mpc.solver.stats()["return_status"]}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(batch, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "batched QP solves/sec (N=16, 4-leg friction cone) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"cfg{cfg} Go2 QP batch (SURVEY.md 8(d)), "
                                   f"{'trot 3Hz/0.6 fixed schedule' if cfg == 1 else 'mixed stance' if cfg == 2 else 'trot+mixed'}",
                       "N": 16, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"instance-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": f"solve_bin_kernel<{[96, 128, 160, 192][q]}>",
                         "kernel_avg_ms": avg_ms, "solves_per_launch": n_in_bin,
                         "bytes_per_solve": BYTES_PER_SOLVE},
            "roofline_compute": {"bound": "mfma", "achieved": achieved_tfs,
                                 "peak": F32_MATRIX_PEAK_TFS, "unit": "TFLOP/s",
                                 "frac": achieved_tfs / F32_MATRIX_PEAK_TFS,
                                 "flops_per_solve": fl_bin / max(n_in_bin, 1)},
            "cpu_baseline": cpu,
            "solved_frac": solved_frac,
            "iters_mean": float(np.mean(iters)),
            "iters_max": int(np.max(iters)),
            "latency_ms_b256": lat_ms,
            "dynamics": dyn,
            "warm_start": warm,
            "tick": tick,
            "leg_controller": leg,
            "closed_loop": loop,
            "config0_api": api,
            "params_override": over or None,
            "bin_ms_per_step": {str(c): round(float(ms_bins[i]) / args.steps, 4)
                                for i, c in enumerate((96, 128, 160, 192))},
            "bin_solves": {str(c): int(np.sum(bins == i)) for i, c in enumerate((96, 128, 160, 192))},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(batch, seconds):
    """Time oracle/osqp_ref (C restatement of the reference's OSQP solve) on host cores."""
    try:
        sys.path.insert(0, str(REPO))
        from oracle import osqp_ref
    except Exception as e:  # pragma: no cover - reported, not fatal
        return {"value": None, "unit": "solves/s", "cores": 0, "kind": "port",
                "sample": f"unavailable: {e}"}
    return osqp_ref.time_baseline(batch, seconds)


if __name__ == "__main__":
    main()
