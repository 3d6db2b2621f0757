#!/usr/bin/env python3
"""bench.py -- batched convex-MPC QP solves/sec on MI355X (BASELINE.json metric).

Headline (BASELINE.json configs[3]): the config-3 workload -- 65,536
synthetic Go2 QP instances, trot (fixed 3 Hz / 0.6 schedule) and mixed stance masks
interleaved -- is ONE global batch sharded over the N ranks (one process per GPU): rank r
solves the contiguous slice [r B/N, (r+1) B/N) of it, resident in its HBM.  One *step* = one
``cmpc_solve`` of every rank's shard; ``value`` = 65,536 x steps / (max over ranks of the
timed region), ``"scaling": "strong"``.

    python bench.py [--gpus N --steps K --warmup W --config 3|2|1 --batch B]

``--gpus N`` (N > 1) without a torch.distributed environment re-launches this script under
``torch.distributed.run`` with N ranks (before anything touches the GPU); under an existing
launcher WORLD_SIZE must equal N.

Also on the line:
  * ``scatter_gather`` (N > 1): the same global batch owned by rank 0 -- one RCCL scatter of
    the input stacks, the solve, one RCCL gather of w per step (cmpc/dist.py);
  * ``weak``: every rank solves the whole 65,536-instance batch (per-GPU work fixed);
  * ``configs`` (N = 1): BASELINE configs 1 (B = 256) and 2 (B = 4,096), plus configs 1 and 2
    at B = 65,536, each timed the same way with its own roofline;
  * ``roofline``: the dominant solve kernel (of the three, cmpc_host.hip) priced against HBM:
    12,264 algorithmic bytes per solve (inputs 10,720 + outputs 1,544) x the solves it
    processed / its average HIP-event duration on its own stream; ``traffic`` = the PMC HBM
    bytes per launch from profiles/;
  * ``cpu_baseline`` (rank 0, N = 1): the oracle's C++ restatement of the reference's OSQP
    path on a bounded sample of the same workload (a reported baseline, not the target);
  * the SURVEY 8(f) objects (N = 1): on-device dynamics, warm start, the on-device tick, the
    leg controller, the closed loop, config 0 through the drop-in API.
"""
from __future__ import annotations

import argparse
import json
import re
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))

METRIC = "batched QP solves/sec (N=16, 4-leg friction cone) at 1/2/4/8 MI355X"
BYTES_IN = 576 + 9216 + 48 + 48 + 768 + 64      # Ad, Bd, gd, x0, xref, contact (N=16, fp32/u8)
BYTES_OUT = 1536 + 4 + 4                         # w, status, iters
BYTES_PER_SOLVE = BYTES_IN + BYTES_OUT           # 12,264
HBM_PEAK_GBS = 8000.0                            # MI355X_MICROARCH.md: 8.0 TB/s spec
F32_MATRIX_PEAK_TFS = 157.3                      # MI355X_MICROARCH.md: dense f32 MFMA peak
POLISH_REFINE = 4                                # SolverParams.polish_refine (default)
GLOBAL_BATCH = {1: 256, 2: 4096, 3: 65536}       # BASELINE.json configs[1..3]
from cmpc._lib import BIN_CAPS, KERNEL_BINS, KERNEL_NAMES  # noqa: E402  (no GPU touched)


def algorithmic_flops(contact, iters, N=16):
    """Algorithmic FP32 work per instance of the path's algorithm: one ADMM and
    one polish factorisation at the instance's free-force count n (condensation
    sum_t 12 m_t^2 + 288 m_{t-1} with m_t = free forces of steps <= t, sweep inverse n^3),
    `iters` ADMM iterations and POLISH_REFINE refinements of symv (2 n^2) + gradient
    (576 N + 48 n).  Counts only the accepted path (no rho refactors, repairs or padding)."""
    st = (contact != 0).reshape(contact.shape[0], 4, -1)
    per_step = 3 * st.sum(1).astype(np.float64)
    m = np.cumsum(per_step, axis=1)
    n = m[:, -1]
    m_prev = np.concatenate([np.zeros((m.shape[0], 1)), m[:, :-1]], axis=1)
    cond = (12.0 * m ** 2 + 288.0 * m_prev).sum(1)
    inv = n ** 3
    symv = 2.0 * n ** 2
    grad = 576.0 * N + 48.0 * n
    it = iters.astype(np.float64)
    return 2.0 * (cond + inv) + it * (symv + grad) + POLISH_REFINE * symv + (POLISH_REFINE + 1) * grad


def bins_of(contact, caps=BIN_CAPS):
    nf = 3 * (contact != 0).reshape(contact.shape[0], -1).sum(1)
    return np.searchsorted(np.asarray(caps), nf)   # first cap >= nf


def kernel_of_bins(bins, kernel_bins=KERNEL_BINS):
    """Solve kernel (timing slot) of each instance's bin (cmpc_host.hip group_first_bin)."""
    k = np.zeros_like(bins)
    for kk, bs in enumerate(kernel_bins):
        for b in bs:
            k[bins == b] = kk
    return k


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=(1, 2, 3),
                    help="headline workload (BASELINE.json configs[1..3]); default 3")
    ap.add_argument("--batch", type=int, default=None,
                    help="GLOBAL batch of the headline (default: the config's own, 3 -> 65536)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-baseline sample (0 = skip)")
    ap.add_argument("--traffic-json", type=str, default=str(REPO / "profiles" / "hbm_traffic.json"),
                    help="PMC-derived HBM bytes per launch of the dominant kernel (profiles/)")
    ap.add_argument("--counters-json", type=str,
                    default=str(REPO / "profiles" / "counters.json"),
                    help="PMC instruction counters of the dominant kernel (profiles/)")
    ap.add_argument("--sub-configs", type=int, default=1,
                    help="N = 1: also time configs 1 / 2 at their own and at 65,536 (0 = skip)")
    ap.add_argument("--scatter-steps", type=int, default=None,
                    help="N > 1: timed steps of the scatter -> solve -> gather variant "
                         "(default --steps; 0 = skip)")
    ap.add_argument("--weak-steps", type=int, default=None,
                    help="timed steps of the weak-scaling variant (default --steps; 0 = skip)")
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
    ap.add_argument("--aux", type=int, default=1,
                    help="0 = headline only (profiling runs): skips every other object")
    ap.add_argument("--seed-offset", type=int, default=0,
                    help="added to the workload seed (experiments: average over batches)")
    ap.add_argument("--param", action="append",
                    default=[kv for kv in os.environ.get("CMPC_PARAMS", "").split(",") if kv],
                    help="SolverParams override key=value (experiments; also $CMPC_PARAMS k=v,k=v)")
    ap.add_argument("--team", type=int, default=-1,
                    help="small-batch team mode for B <= this (cmpc_plan_set_team): -1 auto, 0 off")
    ap.add_argument("--heavy-first", type=int, default=int(os.environ.get("CMPC_HEAVY_FIRST", "-1")),
                    help="NC >= 160 class first for B >= this (cmpc_plan_set_heavy_first): -1 auto, 0 never")
    ap.add_argument("--stance-all", action="store_true",
                    help="experiments: every foot in stance at every step (a standing batch: "
                         "every instance in the NC 192 bin)")
    ap.add_argument("--lib", type=str, default=None,
                    help="alternative build of libcmpc.so (A/B experiments)")
    a = ap.parse_args(argv)
    if not a.aux:
        a.cpu_seconds = 0
        a.sub_configs = a.dynamics_steps = a.warm_steps = a.tick_steps = 0
        a.leg_steps = a.loop_steps = a.api_ticks = 0
        a.scatter_steps = 0 if a.scatter_steps is None else a.scatter_steps
        a.weak_steps = 0 if a.weak_steps is None else a.weak_steps
    if a.scatter_steps is None:
        a.scatter_steps = a.steps
    if a.weak_steps is None:
        a.weak_steps = a.steps
    return a


# ------------------------------------------------------------------------------------------
# process topology
# ------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(n: int, argv) -> int:
    """Start this script under torch.distributed.run with n ranks (child process; this process
    has not touched the GPU) and return its exit code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(Path(__file__).resolve()), *argv]
    return subprocess.call(cmd, env=env)


def topology(args):
    """-> (world, rank, local) from the torch.distributed.run environment, checked against
    --gpus.  Raises SystemExit when they disagree."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                         f"'python bench.py --gpus N' or torchrun --nproc-per-node N ... --gpus N")
    return world, rank, local


def timed_steps(step, steps, warmup, sync, barrier, reduce_max):
    """Run `warmup` untimed steps, then time exactly `steps` steps bracketed by barrier + device
    sync on both sides; -> seconds (max over ranks)."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    return reduce_max(time.perf_counter() - t0)


# ------------------------------------------------------------------------------------------
# GPU measurement helpers
# ------------------------------------------------------------------------------------------
def _counters_of(counters, name):
    """PMC record of kernel `name` in profiles/*_counters.json (keys are rocprof's demangled
    names, e.g. 'void cmpc::solve_group_kernel<128, 96>')."""
    def norm(n):  # (round-4 records name the kernels with a third template flag, <.., .., false>)
        return re.sub(r",(true|false)>", ">", n.replace(" ", ""))
    for k, v in (counters or {}).items():
        if isinstance(v, dict) and norm(k).endswith(norm(name)):
            return v
    return None


def kernel_roofline(plan, B_shard, bins, contact, iters, ms, calls, traffic=None, counters=None,
                    step_ms=None):
    """Rooflines of the solve kernels of the last timed steps: algorithmic bytes of the solves a
    kernel processed / its average HIP-event duration (measured on the stream it runs on).
    Returns (roofline, roofline_compute, roofline_critical):
      * roofline / roofline_compute: the DOMINANT kernel, the one that processes the most solves;
      * roofline_critical: the kernel whose live time sets the step (the longest average launch),
        with its HBM and compute fractions and its share of the step.  With one solve kernel per
        launch (the pair kernel, or the team kernel for small batches) both are the same kernel.
    With PMC counters in profiles/, the compute roofline is the counted MFMA work over the live
    duration; `step` prices every launched kernel together over the whole step."""
    names = plan.solve_kernels(B_shard)
    if names[0] is None:  # an older A/B build without cmpc_plan_solve_kernel
        names = list(KERNEL_NAMES)
    team = names[0].startswith("solve_team")
    nk = len(names)
    live = [k for k in range(nk) if names[k] is not None]
    # one launched kernel (team mode, or a build with one kernel for every bin) solves them all
    kern = np.zeros_like(bins) if len(live) == 1 else kernel_of_bins(bins)
    avg = [ms[k] / max(calls[k], 1) for k in range(nk)]
    n_k = [int(np.sum(kern == k)) for k in range(nk)]
    q = max(live, key=lambda k: n_k[k])          # dominant: most solves
    c = max(live, key=lambda k: avg[k])          # critical: longest live time
    flops = algorithmic_flops(contact, iters)

    def hbm(k):
        achieved = BYTES_PER_SOLVE * n_k[k] / (avg[k] * 1e-3) / 1e9 if avg[k] > 0 else 0.0
        ck = None if team else _counters_of(counters, names[k])
        tr = ck.get("hbm_bytes_per_launch") if ck else (traffic if (k == q and not team) else None)
        tr_raw = ck.get("hbm_bytes_per_launch_raw") if ck else None
        alg = BYTES_PER_SOLVE * n_k[k]
        out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBS, "traffic": tr, "kernel": names[k],
               "kernel_avg_ms": avg[k], "solves_per_launch": n_k[k],
               "bytes_per_solve": BYTES_PER_SOLVE}
        if tr is not None or tr_raw is not None:
            # PMC bytes per launch: `traffic` doubles FETCH_SIZE (the gfx950 correction, exact
            # for 16-B/lane coalesced reads only), `traffic_raw` = FETCH_SIZE + WRITE_SIZE as
            # counted; the kernel's narrow / scratch loads put the true HBM bytes between them
            out.update(traffic_raw=tr_raw, algorithmic_bytes_per_launch=alg,
                       traffic_over_algorithmic=(tr / alg if tr and alg else None),
                       traffic_raw_over_algorithmic=(tr_raw / alg if tr_raw and alg else None))
        return out

    def compute(k):
        fl = float(flops[kern == k].sum())
        tfs = fl / (avg[k] * 1e-3) / 1e12 if avg[k] > 0 else 0.0
        comp = {"bound": "mfma", "achieved": tfs, "peak": F32_MATRIX_PEAK_TFS, "unit": "TFLOP/s",
                "frac": tfs / F32_MATRIX_PEAK_TFS, "kernel": names[k],
                "basis": "algorithmic FLOP model (bench.algorithmic_flops)",
                "flops_per_solve": fl / max(n_k[k], 1)}
        ck = None if team else _counters_of(counters, names[k])
        if ck and ck.get("SQ_INSTS_MFMA") and avg[k] > 0:
            # counted matrix work of this kernel per launch (PMC, profiles/) over its live duration
            ach = ck["SQ_INSTS_MFMA"] * 2048.0 / (avg[k] * 1e-3) / 1e12
            comp.update(model_achieved=tfs, model_frac=tfs / F32_MATRIX_PEAK_TFS, achieved=ach,
                        frac=ach / F32_MATRIX_PEAK_TFS,
                        basis="SQ_INSTS_MFMA x 2048 FLOP (v_mfma_f32_16x16x4_f32) per launch from "
                              "the profiles/ counters / live kernel time",
                        mfma_per_launch=ck["SQ_INSTS_MFMA"], mfma_busy_frac_pmc=ck.get("mfma_busy_frac"))
        return comp

    roof = hbm(q)
    roof.update(kernel_avg_ms_all={names[k]: avg[k] for k in live},
                solves_per_kernel={names[k]: n_k[k] for k in live})
    comp = compute(q)
    crit = hbm(c)
    crit["compute"] = compute(c)
    crit["step_share"] = avg[c] / step_ms if step_ms else None
    crit["same_as_dominant"] = c == q
    if step_ms and not team:
        # every launched solve kernel together over the step
        mf = [(_counters_of(counters, names[k]) or {}).get("SQ_INSTS_MFMA") for k in live]
        st = {"step_ms": step_ms, "solves": int(sum(n_k[k] for k in live)),
              "hbm_achieved_GBs": BYTES_PER_SOLVE * sum(n_k[k] for k in live) / (step_ms * 1e-3) / 1e9}
        st["hbm_frac"] = st["hbm_achieved_GBs"] / HBM_PEAK_GBS
        if all(m for m, k in zip(mf, live) if n_k[k] > 0) and any(mf):
            tf = sum(m for m in mf if m) * 2048.0 / (step_ms * 1e-3) / 1e12
            st.update(mfma_achieved_TFs=tf, mfma_frac=tf / F32_MATRIX_PEAK_TFS,
                      mfma_basis="SQ_INSTS_MFMA of the launched kernels (profiles/ counters)")
        comp["step"] = st
    return roof, comp, crit


def load_json(path):
    if path and Path(path).exists():
        try:
            return json.loads(Path(path).read_text())
        except Exception:
            return None
    return None


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args.gpus, argv))
    world, rank, local = topology(args)

    import torch
    import torch.distributed as dist
    if os.environ.get("CMPC_BENCH_DRYRUN") == "1":
        return dry_run(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.lib:
        from cmpc import _lib
        _lib._lib = _lib.load(args.lib)
    from cmpc import Plan, SolverParams, to_device_batch, synth
    from cmpc import dist as cdist

    def sync():
        torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def reduce_max(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def reduce_sum_int(x):
        if world == 1:
            return int(x)
        t = torch.tensor([x], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    over = {}
    for kv in args.param:
        k, v = kv.split("=")
        over[k] = type(getattr(SolverParams, k))(float(v) if "." in v or "e" in v else int(v))

    cfg = args.config
    GB = args.batch or GLOBAL_BATCH[cfg]
    if cfg == 3:
        full = synth.make_config(3, B=GB)
    else:
        full = synth.make_batch(GB, seed=synth.CONFIGS[cfg]["seed"] + args.seed_offset,
                                mixed=synth.CONFIGS[cfg]["mixed"])
    if args.stance_all:
        full["contact"] = np.ones_like(full["contact"])
    lo, hi = cdist.shard_bounds(GB, rank, world)
    shard = {k: full[k][lo:hi] for k in cdist.FIELDS}
    Bs = hi - lo
    max_b = max(GB if args.weak_steps > 0 else Bs, 65536 if (world == 1 and args.sub_configs) else 0)
    plan = Plan(SolverParams(max_batch=max_b, **over), device=dev)
    if args.team != -1 and hasattr(plan.lib, "cmpc_plan_set_team"):
        plan.set_team(args.team)
    if args.heavy_first != -1 and hasattr(plan.lib, "cmpc_plan_set_heavy_first"):
        plan.set_heavy_first(args.heavy_first)
    stream = torch.cuda.current_stream(dev)
    d = to_device_batch(shard, dev)
    w = torch.empty((Bs, 24 * 16), dtype=torch.float32, device=dev)
    st = torch.empty((Bs,), dtype=torch.int32, device=dev)
    it = torch.empty((Bs,), dtype=torch.int32, device=dev)

    def step():
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                   out=(w, st, it), stream=stream)

    # ---- headline: strong scaling of the config's global batch over the ranks ----
    for _ in range(args.warmup):
        step()
    sync()
    plan.timing_read()
    plan.stats(reset=True)
    plan.set_timing(True)
    elapsed = timed_steps(step, args.steps, 0, sync, barrier, reduce_max)
    plan.set_timing(False)
    ms_k, calls_k = plan.timing_read()
    acc = plan.stats(reset=True)   # (after the timed region: it synchronises)
    n_ranks = reduce_sum_int(1)
    # acceptance statistics of the timed steps, summed over the ranks, per step (cmpc_plan_stats)
    acceptance = {k: (reduce_sum_int(v) / args.steps if v is not None else None)
                  for k, v in acc.items()}
    solved = reduce_sum_int(int((st == 1).sum().item()))
    status = st.cpu().numpy()
    iters = it.cpu().numpy()
    value = GB * args.steps / elapsed
    bins = bins_of(shard["contact"])
    traffic_j = load_json(args.traffic_json)
    traffic = traffic_j.get("hbm_bytes_per_launch") if traffic_j else None
    # the PMC counters were collected on one full config-3 launch (65,536 solves on one GPU):
    # per-launch counts apply only to that workload
    counters = load_json(args.counters_json) if (args.config == 3 and Bs == 65536) else None
    roof, roof_c, roof_crit = kernel_roofline(plan, Bs, bins, shard["contact"], iters, ms_k,
                                              calls_k, traffic, counters,
                                              step_ms=1e3 * elapsed / args.steps)

    # ---- N > 1: scatter from rank 0 -> solve -> gather to rank 0 (RCCL over xGMI) ----
    scat = None
    if world > 1 and args.scatter_steps > 0:
        src = to_device_batch({k: full[k] for k in cdist.FIELDS}, dev) if rank == 0 else None
        holder = {}

        def sg_step():
            mine = cdist.scatter_batch(src, GB, 16, dev)
            ww, ss, ii = plan.solve(mine["Ad"], mine["Bd"], mine["gd"], mine["x0"], mine["xref"],
                                    mine["contact"], stream=stream)
            holder["w"] = cdist.gather_solutions(ww, GB)
        el = timed_steps(sg_step, args.scatter_steps, 2, sync, barrier, reduce_max)
        ok = True
        if rank == 0:   # the gathered solutions are the headline's, instance by instance
            ok = bool(holder["w"].shape == (GB, 384))
        scat = {"solves_per_s": GB * args.scatter_steps / el,
                "ms_per_step": el / args.scatter_steps * 1e3,
                "steps": args.scatter_steps,
                "comm": "dist.scatter of the 6 input stacks (10,720 B/instance) + dist.gather of "
                        "w (1,536 B/instance) from/to rank 0 over RCCL, per step",
                "gathered_shape_ok": ok}
        del src

    # ---- weak scaling: every rank solves the whole global batch ----
    weak = None
    if args.weak_steps > 0 and (world > 1 or GB != Bs):
        dfull = to_device_batch({k: full[k] for k in cdist.FIELDS}, dev)
        wf = torch.empty((GB, 384), dtype=torch.float32, device=dev)
        sf = torch.empty((GB,), dtype=torch.int32, device=dev)
        itf = torch.empty((GB,), dtype=torch.int32, device=dev)

        def wk_step():
            plan.solve(dfull["Ad"], dfull["Bd"], dfull["gd"], dfull["x0"], dfull["xref"],
                       dfull["contact"], out=(wf, sf, itf), stream=stream)
        el = timed_steps(wk_step, args.weak_steps, 2, sync, barrier, reduce_max)
        weak = {"solves_per_s": GB * world * args.weak_steps / el,
                "ms_per_step": el / args.weak_steps * 1e3, "batch_per_gpu": GB,
                "scaling": "weak"}
        del dfull, wf, sf, itf

    # ---- N = 1: BASELINE configs 1 and 2 at their own batch, and configs 1 / 2 at 65,536 ----
    configs = None
    if world == 1 and args.sub_configs:
        configs = {}
        for name, c, B in (("config1_b256", 1, 256), ("config2_b4096", 2, 4096),
                           ("config1_b65536", 1, 65536), ("config2_b65536", 2, 65536)):
            b = synth.make_batch(B, seed=synth.CONFIGS[c]["seed"] + args.seed_offset,
                                 mixed=synth.CONFIGS[c]["mixed"])
            db = to_device_batch(b, dev)
            wb = torch.empty((B, 384), dtype=torch.float32, device=dev)
            sb = torch.empty((B,), dtype=torch.int32, device=dev)
            ib = torch.empty((B,), dtype=torch.int32, device=dev)

            def c_step():
                plan.solve(db["Ad"], db["Bd"], db["gd"], db["x0"], db["xref"], db["contact"],
                           out=(wb, sb, ib), stream=stream)
            ksteps = 50 if B <= 4096 else args.steps
            for _ in range(3):
                c_step()
            sync()
            plan.timing_read()
            plan.set_timing(True)
            el = timed_steps(c_step, ksteps, 0, sync, barrier, reduce_max)
            plan.set_timing(False)
            mk, ck = plan.timing_read()
            itb = ib.cpu().numpy()
            r, rc, rcrit = kernel_roofline(plan, B, bins_of(b["contact"]), b["contact"], itb, mk,
                                           ck, step_ms=el / ksteps * 1e3)
            configs[name] = {"solves_per_s": B * ksteps / el, "ms_per_step": el / ksteps * 1e3,
                             "batch": B, "steps": ksteps,
                             "solved_frac": float((sb == 1).float().mean().item()),
                             "iters_mean": float(itb.mean()), "iters_max": int(itb.max()),
                             "roofline": {k: r[k] for k in ("achieved", "frac", "kernel",
                                                            "kernel_avg_ms", "kernel_avg_ms_all",
                                                            "solves_per_kernel")},
                             "roofline_compute_frac": rc["frac"],
                             "roofline_critical": {k: rcrit[k] for k in ("kernel", "kernel_avg_ms",
                                                                         "frac", "step_share")}}
            del db, wb, sb, ib

    aux = {}
    if world == 1:
        if args.aux:
            aux["shard_rehearsal"] = shard_rehearsal(plan, d, GB, stream, torch)
        aux.update(aux_objects(args, plan, full, dev, stream, torch))

    cpu = None
    odist = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(full, args.cpu_seconds)
        w_osqp = cpu.pop("_w", None)
        if w_osqp is not None:
            odist = osqp_distance(full, w.cpu().numpy(), w_osqp, cpu["cores"])

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": (f"BASELINE config {cfg}: {GB} Go2 QP instances (N=16) "
                                    + ("trot 3Hz/0.6 + mixed stance masks interleaved"
                                       if cfg == 3 else "trot 3Hz/0.6 fixed schedule" if cfg == 1
                                       else "mixed stance masks")
                                    + (" (EXPERIMENT: all feet in stance)" if args.stance_all else "")
                                    + f", one global batch sharded over {world} rank(s), "
                                      "inputs resident in HBM"),
                       "N": 16, "global_batch": GB, "batch_per_gpu": Bs,
                       "parallelism": f"instance-sharded x{world} (contiguous slices, no "
                                      "data-path collective)"},
            "ranks_reporting": n_ranks,
            "roofline": roof,
            "roofline_compute": roof_c,
            "roofline_critical": roof_crit,
            "cpu_baseline": cpu,
            "osqp_distance": odist,
            "solved_frac": solved / GB,
            "iters_mean": float(np.mean(iters)),
            "iters_max": int(np.max(iters)),
            "status_counts": {str(s): int(np.sum(status == s)) for s in np.unique(status)},
            "acceptance_per_step": acceptance,
            "bin_solves": {str(c): int(np.sum(bins == i)) for i, c in enumerate(BIN_CAPS)},
            "scatter_gather": scat,
            "weak": weak,
            "configs": configs,
            **aux,
            "params_override": over or None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dry_run(args, world, rank):
    """CMPC_BENCH_DRYRUN=1 (CPU tests): the rank / shard logic of the headline with the solve
    stubbed -- gloo instead of RCCL, no device.  Rank 0 prints the world size all ranks agree
    on, each rank's slice of the global batch and the step timing's max-over-ranks."""
    import torch
    import torch.distributed as dist
    from cmpc import dist as cdist
    if world > 1:
        dist.init_process_group("gloo")
    GB = args.batch or GLOBAL_BATCH[args.config]
    lo, hi = cdist.shard_bounds(GB, rank, world)

    def reduce_max(x):
        t = torch.tensor([x], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier():
        if world > 1:
            dist.barrier()
    work = {"n": 0}

    def step():   # stub solve: touch the shard
        work["n"] += hi - lo
    el = timed_steps(step, args.steps, args.warmup, lambda: None, barrier, reduce_max)
    t = torch.tensor([1, hi - lo, work["n"]], dtype=torch.int64)
    spans = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_gather(spans, torch.tensor([lo, hi], dtype=torch.int64))
    else:
        spans = [torch.tensor([lo, hi])]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_reporting": int(t[0]), "global_batch": GB,
                          "solved_per_step": int(t[1]), "stub_work": int(t[2]),
                          "spans": [s.tolist() for s in spans], "elapsed_max": el,
                          "steps": args.steps, "warmup": args.warmup}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def aux_objects(args, plan, full, dev, stream, torch):
    """SURVEY.md 8(f) objects on one GPU: each times its own component on a 65,536-robot batch
    (the headline's instances where they apply)."""
    from cmpc import to_device_batch, synth
    out = {}
    B = min(65536, full["Ad"].shape[0])
    batch = {k: (v[:B] if isinstance(v, np.ndarray) else v) for k, v in full.items()}
    d = to_device_batch(batch, dev)
    w = torch.empty((B, 384), dtype=torch.float32, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731

    # 8(f) row 1: the discrete dynamics built on the device -- its own HBM roofline, and the
    # fused per-tick throughput build + solve
    if args.dynamics_steps > 0:
        N = 16
        dm = {k: torch.as_tensor(batch[k], dtype=torch.float32).contiguous().to(dev)
              for k in ("m", "I_world", "r_legs")}
        dt = float(batch["dt"])
        outs = (torch.empty_like(d["Ad"]), torch.empty_like(d["Bd"]), torch.empty_like(d["gd"]))
        for _ in range(2):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
        sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.dynamics_steps):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
        e1.record(stream)
        sync()
        dyn_ms = e0.elapsed_time(e1) / args.dynamics_steps
        dyn_bytes = B * (4 + 36 + N * 48 + N * 48 + 576 + N * 576 + 48)
        t0f = time.perf_counter()
        for _ in range(args.dynamics_steps):
            plan.build_dynamics(dm["m"], dm["I_world"], dm["r_legs"], d["xref"], dt, out=outs,
                                stream=stream)
            plan.solve(outs[0], outs[1], outs[2], d["x0"], d["xref"], d["contact"],
                       out=(w, st, it), stream=stream)
        sync()
        fused = B * args.dynamics_steps / (time.perf_counter() - t0f)
        gbs = dyn_bytes / (dyn_ms * 1e-3) / 1e9
        out["dynamics"] = {"kernel": "dynamics_kernel", "ms_per_step": dyn_ms,
                           "robots_per_s": B / (dyn_ms * 1e-3),
                           "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                                        "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                        "bytes_per_robot": dyn_bytes // B},
                           "fused_build_and_solve_per_s": fused}

    # 8(f) row 4: warm start (centroidal_mpc.py:91-95).  Next-tick proxy: the state moves
    # (x0 + noise), reference and gait stay; every warm step starts from the previous tick's
    # (w, y).  Cold and warm solves of the same next-tick batch, same timing method.
    if args.warm_steps > 0:
        y0 = torch.empty((B, 12 * 16), dtype=torch.float32, device=dev)
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"],
                   out=(w, st, it), stream=stream, y_out=y0)
        w0 = w.clone()
        g = torch.Generator(device=dev).manual_seed(1234)
        sc = torch.tensor([2e-3] * 6 + [2e-2] * 6, device=dev)
        d2 = dict(d)
        d2["x0"] = (d["x0"] + torch.randn(d["x0"].shape, generator=g, device=dev) * sc).contiguous()
        y1 = torch.empty_like(y0)

        def timed(warm_on):
            kw = dict(w_init=w0, y_init=y0, y_out=y1) if warm_on else {}
            for _ in range(2):
                plan.solve(d2["Ad"], d2["Bd"], d2["gd"], d2["x0"], d2["xref"], d2["contact"],
                           out=(w, st, it), stream=stream, **kw)
            sync()
            ta = time.perf_counter()
            for _ in range(args.warm_steps):
                plan.solve(d2["Ad"], d2["Bd"], d2["gd"], d2["x0"], d2["xref"], d2["contact"],
                           out=(w, st, it), stream=stream, **kw)
            sync()
            el = time.perf_counter() - ta
            itn = it.cpu().numpy()
            return (B * args.warm_steps / el, float(itn.mean()), (st == 1).float().mean().item(),
                    int(itn.max()), float(np.percentile(itn, 99.9)))
        cold_rate, cold_it, cold_ok, cold_max, cold_p = timed(False)
        warm_rate, warm_it, warm_ok, warm_max, warm_p = timed(True)
        out["warm_start"] = {
            "scenario": "next tick: x0 + N(0, 2e-3 pos/rpy, 2e-2 vel/omega); warm from the "
                        "previous tick's (w, y_out), cmpc_solve_warm",
            "solves_per_s_warm": warm_rate, "solves_per_s_cold": cold_rate,
            "speedup": warm_rate / cold_rate, "iters_mean_warm": warm_it,
            "iters_mean_cold": cold_it, "solved_frac_warm": warm_ok,
            "solved_frac_cold": cold_ok, "iters_max_warm": warm_max,
            "iters_max_cold": cold_max, "iters_p999_warm": warm_p, "iters_p999_cold": cold_p}

    # 8(f) row 2: the whole tick on the device -- reference trajectory, contact table and foot
    # levers (cmpc_generate_traj, com_trajectory.py:27-207) -> discrete dynamics -> solve.
    if args.tick_steps > 0:
        tk = synth.make_tick_inputs(B, seed=synth.CONFIGS[2]["seed"] + 500, mixed=True)
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
        sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.tick_steps):
            gen()
        e1.record(stream)
        sync()
        tr_ms = e0.elapsed_time(e1) / args.tick_steps
        tr_bytes = 48 + 24 + 16 + 8 + 48 + 48 + N * 48 + 4 * N + N * 48 + 24   # in + out per robot
        t0t = time.perf_counter()
        for _ in range(args.tick_steps):
            full_tick()
        sync()
        tick_rate = B * args.tick_steps / (time.perf_counter() - t0t)
        td["pos_des"].copy_(pd0)
        tick_it = it.cpu().numpy()
        gbs_t = tr_bytes * B / (tr_ms * 1e-3) / 1e9
        out["tick"] = {"kernel": "traj_group_kernel", "ms_per_step": tr_ms,
                       "roofline": {"bound": "hbm", "achieved": gbs_t, "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": gbs_t / HBM_PEAK_GBS,
                                    "bytes_per_robot": tr_bytes},
                       "full_tick_per_s": tick_rate,
                       "full_tick": "generate_traj + build_dynamics + cold solve, all on the "
                                    "device (mixed gaits)",
                       "solved_frac": float((st == 1).float().mean().item()),
                       "iters_mean": float(tick_it.mean())}

    # 8(f) row 3: the consumer of U[:, 0] -- the 1 kHz leg controller (leg_controller.py:43-112)
    # for every robot of the batch, with synthetic Pinocchio quantities and the solver's forces.
    if args.leg_steps > 0:
        from cmpc import leg_state
        gl = torch.Generator(device=dev).manual_seed(77)
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
        sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.leg_steps):
            tl.add_(0.001)
            leg_step()
        e1.record(stream)
        sync()
        leg_ms = e0.elapsed_time(e1) / args.leg_steps
        leg_bytes = (8 + 48 + 48 + 288 + 1728 + 2592 + 1728 + 96 + 144 + 96 * 3 + 128 + 256
                     + 96 + 256)
        gbs_l = leg_bytes * B / (leg_ms * 1e-3) / 1e9
        out["leg_controller"] = {
            "kernel": "leg_kernel", "ms_per_step": leg_ms, "robots_per_s": B / (leg_ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": gbs_l, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs_l / HBM_PEAK_GBS, "bytes_per_robot": leg_bytes},
            "note": "includes the small add_ on t per step; trot gait, 2 legs swing most ticks"}
        del li, Ml

    # BASELINE config 4 shape: robots in closed loop, every MPC tick on the device
    # (generate_traj -> build_dynamics -> warm solve -> SRB plant for 20 leg ticks), recorded
    # once as a HIP graph and replayed.  MuJoCo is absent: the plant is cmpc_srb_step's stand-in.
    if args.loop_steps > 0:
        from cmpc.closed_loop import ClosedLoop
        loop = {"plant": "cmpc_srb_step single-rigid-body stand-in (MuJoCo absent)",
                "mpc_dt_s": 1 / 48}
        for nb in (1024, B):
            # eager and graph replay on the same tick sequence: two loops from the same seed,
            # 5 untimed ticks each (the graph's capture records tick 5, its first replay runs
            # it), then ticks 6 .. 5 + loop_steps timed
            rg = np.random.default_rng(100)
            cmd = np.stack([rg.uniform(-0.5, 0.5, nb), rg.uniform(-0.2, 0.2, nb),
                            np.full(nb, 0.27), rg.uniform(-1, 1, nb)], 1)
            rate = {}
            for mode in ("eager", "graph"):
                cl = ClosedLoop(nb, plan=plan, seed=0)
                cl.set_command(cmd)
                for _ in range(4):
                    cl.tick()
                if mode == "graph":
                    cl.capture()
                cl.tick()
                sync()
                t0 = time.perf_counter()
                for _ in range(args.loop_steps):
                    cl.tick()
                sync()
                el = time.perf_counter() - t0
                rate[mode] = (nb * args.loop_steps / el, el / args.loop_steps * 1e3)
                if mode == "graph":
                    loop[f"robots_{nb}"] = {
                        "robot_ticks_per_s_graph": rate["graph"][0],
                        "ms_per_tick_graph": rate["graph"][1],
                        "robot_ticks_per_s_eager": rate["eager"][0],
                        "ms_per_tick_eager": rate["eager"][1],
                        "ticks": f"6..{5 + args.loop_steps} in both modes",
                        "solved_frac": float((cl.status == 1).float().mean().item()),
                        "iters_mean": float(cl.iters.float().mean().item()),
                        "com_z_min": float(cl.x[:, 2].min().item())}
                del cl
        out["closed_loop"] = loop

    # BASELINE config 0: one robot through the reference's own API (CentroidalMPC.solve_QP, the
    # drop-in of centroidal_mpc.py), warm-started every tick as the reference does; the
    # reference budget per MPC tick is MPC_DT = 20.8 ms (test_MPC.py:67-68).
    if args.api_ticks > 0:
        import contextlib
        import types
        from centroidal_mpc import CentroidalMPC
        one = synth.make_batch(1, seed=0)
        traj = types.SimpleNamespace(
            N=16, Ad=one["Ad"][0], Bd=one["Bd"][0], gd=one["gd"][0].reshape(12, 1),
            initial_x_vec=one["x0"][0].reshape(12, 1), contact_table=one["contact"][0].astype(np.int32),
            compute_x_ref_vec=lambda: one["xref"][0].T.copy())
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
        out["config0_api"] = {
            "path": "CentroidalMPC(go2, traj).solve_QP -> sol['x'].full(), 1 robot, warm",
            "solve_time_ms": float(np.median(st_ms)), "update_time_ms": float(np.median(up_ms)),
            "wall_ms_per_tick": float(np.median(wall)), "mpc_dt_budget_ms": 1e3 / 48,
            "return_status": mpc.solver.stats()["return_status"]}
    return out


def _rel_u(wa, wb, N=16):
    """max_k,leg |U_a - U_b| / max |U_b| per instance (the parity metric of tests/)."""
    ua, ub = np.asarray(wa, np.float64)[:, 12 * N:], np.asarray(wb, np.float64)[:, 12 * N:]
    return np.abs(ua - ub).max(1) / np.maximum(np.abs(ub).max(1), 1e-12)


def osqp_distance(full, w_gpu, w_osqp, cores, n_tight=256):
    """Informational: how far this solver's forces are from what the
    reference's OSQP solve returns, on the cpu_baseline sample, and how far that OSQP output
    (reference OPTS, eps 1e-4) is from the optimum -- the optimum being the same restatement run
    to eps 1e-10 on the first n_tight instances.  The parity bar (tests/) is against the
    KKT-certified optimum."""
    from oracle import osqp_ref
    n = w_osqp.shape[0]
    wg = w_gpu[:n]
    m = min(n, n_tight)
    sub = {k: v[:m] for k, v in full.items() if isinstance(v, np.ndarray)}
    rt = osqp_ref.solve_batch(sub, threads=cores, settings=osqp_ref.tight_settings())
    ok = rt["status"] == 1

    def stats(e):
        return {"median": float(np.median(e)), "max": float(np.max(e)),
                "p90": float(np.percentile(e, 90))} if len(e) else None
    return {"metric": "max |U_a - U_b| / max |U_b| per instance (forces u_0..u_15)",
            "gpu_vs_osqp_ref": stats(_rel_u(wg, w_osqp)), "sample": int(n),
            "osqp_ref_vs_optimum": stats(_rel_u(w_osqp[:m], rt["w"])[ok]),
            "gpu_vs_optimum": stats(_rel_u(wg[:m], rt["w"])[ok]),
            "optimum_sample": int(m), "optimum_converged_frac": float(ok.mean()),
            "optimum": "oracle/osqp_ref.cpp at eps 1e-10 (converges to the KKT-certified optimum)",
            "osqp_ref": "oracle/osqp_ref.cpp with the reference OPTS (centroidal_mpc.py:20-36)"}


def shard_rehearsal(plan, d, GB, stream, torch, reps=5):
    """Strong-scaling rehearsal on one GPU: every rank's contiguous shard of
    the global batch (cmpc.dist.shard_bounds) solved alone, median of `reps` HIP-event-timed
    solves each.  An N-GPU step lasts as long as its slowest shard, so the predicted speedup at
    N is (N = 1 time) / max over the N shards."""
    from cmpc.dist import shard_bounds
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {"method": "each shard of the config's global batch solved alone on this GPU, median "
                     f"of {reps}; step(N) = max over the N shards", "N": {}}
    base = None
    for R in (1, 2, 4, 8):
        ms = []
        for r in range(R):
            lo, hi = shard_bounds(GB, r, R)
            args = [d[k][lo:hi] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")]
            plan.solve(*args, stream=stream)
            t = []
            for _ in range(reps):
                e0.record(stream)
                plan.solve(*args, stream=stream)
                e1.record(stream)
                e1.synchronize()
                t.append(e0.elapsed_time(e1))
            ms.append(float(np.median(t)))
        step = max(ms)
        base = step if base is None else base
        out["N"][str(R)] = {"shard_ms": ms, "step_ms": step, "predicted_speedup": base / step,
                            "predicted_solves_per_s": GB / (step * 1e-3)}
    return out


def cpu_baseline(batch, seconds):
    """Time oracle/osqp_ref (C++ restatement of the reference's OSQP solve) on host cores."""
    try:
        sys.path.insert(0, str(REPO))
        from oracle import osqp_ref
    except Exception as e:  # pragma: no cover - reported, not fatal
        return {"value": None, "unit": "solves/s", "cores": 0, "kind": "port",
                "sample": f"unavailable: {e}"}
    return osqp_ref.time_baseline(batch, seconds)


if __name__ == "__main__":
    main()
