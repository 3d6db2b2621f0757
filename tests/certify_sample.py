"""Parity survey beyond the committed fixtures (test infrastructure, not collected by pytest):
whole batches solved by the HIP path, then EVERY instance certified on the CPU against its
KKT-certified optimum (oracle/active_set.py, the certificate of the golden fixtures) and the
distribution of max|dU| / max|U| reported per batch.

    python tests/certify_sample.py gpu [--sets a,b]   # GPU box: solve, keep U in $SURVEY_DIR
    python tests/certify_sample.py cpu [--sets a,b]   # certify (GPU box or here; 16 processes)

The two phases are separate processes: the certifying pool never shares a process with the
GPU.  Sets (the parity bar is 1e-4 on every status-1 instance):
  cfg2_next_cold   test_warm_next_tick's batch: config 2 at 4,096 (seed 2), x0 moved
                   (synth.next_tick), cold
  cfg2_next_warm   the same problems warm-started from the previous tick's (w, y_out)
  cfg2_next_ref    the same, warm-started from the previous tick's reference multipliers
                   (cmpc_solve_ref: w_init + lam_init)
  cfg2_4096        BASELINE config 2 at its own 4,096, cold
  cfg1_256         BASELINE config 1 at its own 256 (team kernel), cold
  cfg3_65536       the headline batch (config 3, 65,536), cold, every instance
  cfg3_next_warm   the headline batch's next tick warm-started from its (w, y_out), every instance
  cfg2_65536       config 2's distribution at 65,536, cold, every instance
  (--sets with EXTRA: mixed_s11_65536, trot_s12_65536 cold and mixed_s13_next_warm, fresh seeds)
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import get_context
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tests"), str(REPO), str(REPO / "convex-mpc-unitree-go2_amd")]
DIR = Path(os.environ.get("SURVEY_DIR", "/tmp/cmpc_survey"))
ALL = ("cfg2_next_cold", "cfg2_next_warm", "cfg2_next_ref", "cfg2_4096", "cfg1_256",
       "cfg3_65536", "cfg3_next_warm", "cfg2_65536")
# fresh seeds (round 6): problems no test, fixture or tuning run has seen
EXTRA = ("mixed_s11_65536", "trot_s12_65536", "mixed_s13_next_warm")


def batch_of(name):
    from cmpc import synth
    if name.startswith("cfg2_next"):
        b = synth.make_config(2, B=4096)
        return synth.next_tick(b), (None if name.endswith("_cold") else b)
    if name == "cfg2_4096":
        return synth.make_config(2, B=4096), None
    if name == "cfg1_256":
        return synth.make_config(1, B=256), None
    if name == "cfg3_65536":
        return synth.make_config(3), None
    if name == "cfg3_next_warm":
        return synth.next_tick(synth.make_config(3)), synth.make_config(3)
    if name == "cfg2_65536":
        return synth.make_config(2, B=65536), None
    if name == "mixed_s11_65536":
        return synth.make_batch(65536, 11, mixed=True), None
    if name == "trot_s12_65536":
        return synth.make_batch(65536, 12, mixed=False), None
    if name == "mixed_s13_next_warm":
        b = synth.make_batch(65536, 13, mixed=True)
        return synth.next_tick(b), b
    raise KeyError(name)


def gpu(sets, lib=None, params=()):
    import torch
    from cmpc import _lib
    if lib:  # a variant build (A/B surveys)
        _lib._lib = _lib.load(lib)
    from cmpc import Plan, SolverParams, to_device_batch
    DIR.mkdir(parents=True, exist_ok=True)
    over = {k: type(getattr(SolverParams, k))(float(v)) for k, v in (a.split("=") for a in params)}
    plan = Plan(SolverParams(max_batch=65536, **over))
    for name in sets:
        t0 = time.time()
        b, prev = batch_of(name)
        d = to_device_batch(b)
        if prev is None:
            w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
        else:
            p = to_device_batch(prev)
            if name.endswith("_ref"):
                w0, _, _, lam0 = plan.solve(p["Ad"], p["Bd"], p["gd"], p["x0"], p["xref"],
                                            p["contact"], lam_out=True)
                w, st, it, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"],
                                          d["contact"], w_init=w0, lam_init=lam0, lam_out=True)
            else:
                w0, _, _, y0 = plan.solve(p["Ad"], p["Bd"], p["gd"], p["x0"], p["xref"],
                                          p["contact"], y_out=True)
                w, st, it, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"],
                                          d["contact"], w_init=w0, y_init=y0, y_out=True)
        torch.cuda.synchronize()
        N = 16
        np.savez(DIR / f"{name}.npz", U=w[:, 12 * N:].cpu().numpy(), st=st.cpu().numpy(),
                 it=it.cpu().numpy())
        print(f"{name}: solved {len(st)} in {time.time() - t0:.1f} s", flush=True)


_B = None
_U = None


def _one_thread():
    """Pool workers: one BLAS thread each (the box sets 16 threads per process)."""
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def _one(i):
    from oracle import active_set, mpc_qp
    b = _B
    qp = mpc_qp.build_qp(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], b["xref"][i].T,
                         b["contact"][i])
    U = _U[i].astype(np.float64)
    X = mpc_qp.rollout(b["Ad"][i], b["Bd"][i], b["gd"][i], b["x0"][i], U.reshape(-1, 12))
    r = active_set.certified_optimum(qp, np.concatenate([X.reshape(-1), U]))
    Uo = r["w"][12 * qp["N"]:]
    err = float(np.max(np.abs(U - Uo)) / max(np.max(np.abs(Uo)), 1e-12))
    return err, max(r["kkt"].values()), r["steps"], Uo.astype(np.float32)


def cpu(sets, procs, report):
    global _B, _U
    lines, worst_all = [], {}
    Path(report).parent.mkdir(parents=True, exist_ok=True)
    for name in sets:
        t0 = time.time()
        first = len(lines)
        z = dict(np.load(DIR / f"{name}.npz"))
        _B, _ = batch_of(name)
        _U = z["U"]
        B = len(z["st"])
        res = []
        with get_context("fork").Pool(procs, initializer=_one_thread) as pool:
            for k, r in enumerate(pool.imap(_one, range(B), chunksize=64)):
                res.append(r)
                if (k + 1) % 8192 == 0:
                    print(f"  {name}: {k + 1}/{B} certified ({time.time() - t0:.0f} s)", flush=True)
        err = np.array([r[0] for r in res])
        kkt = np.array([r[1] for r in res])
        steps = np.array([r[2] for r in res])
        st, it = z["st"], z["it"]
        ok = st == 1
        nf = 3 * (_B["contact"] != 0).reshape(B, -1).sum(1)
        e1 = err[ok]
        # a reference whose certificate failed (kkt > CERT_TOL: the seeded active-set steps did
        # not close and the interior point stopped short) is no optimum to measure against:
        # counted and named on their own line, never folded into "certified"
        from oracle.active_set import CERT_TOL
        uncert = kkt > CERT_TOL
        head = ("every one certified" if not uncert.any() else
                f"{int((~uncert).sum())} certified, {int(uncert.sum())} NOT certified")
        lines.append(f"{name}: {B} instances, {head} (max KKT residual {(kkt[~uncert].max() if (~uncert).any() else np.nan):.1e}, "
                     f"active-set steps from the GPU's faces: 0 {np.mean(steps == 0):.4f}, "
                     f"1 {np.mean(steps == 1):.4f}, >1 {np.mean(steps > 1):.4f}, "
                     f"fallback {int(np.sum(steps < 0))})")
        if uncert.any():
            bad = np.flatnonzero(uncert)[:8]
            lines.append("  NOT certified (reference KKT residual, error against it): " +
                         ", ".join(f"{int(i)} ({kkt[i]:.1e}, {err[i]:.2e})" for i in bad))
        lines.append(f"  status: " + ", ".join(f"{s}: {int(np.sum(st == s))}" for s in np.unique(st)) +
                     f"; iterations mean {it.mean():.2f} max {it.max()}")
        lines.append(f"  max|dU|/max|U| over status 1: median {np.median(e1):.2e}  p99 {np.quantile(e1, .99):.2e}"
                     f"  p99.9 {np.quantile(e1, .999):.2e}  max {e1.max():.2e};  above 1e-4: "
                     f"{int(np.sum(e1 > 1e-4))}, above 5e-5: {int(np.sum(e1 > 5e-5))}")
        if (~ok).any():
            lines.append(f"  not status 1: max error {err[~ok].max():.2e} over {int((~ok).sum())}")
        for q, cap in enumerate((96, 128, 144, 160, 192)):
            lo = (0, 96, 128, 144, 160)[q]
            m = ok & (nf > lo) & (nf <= cap)
            if m.any():
                lines.append(f"    bin NC {cap:3d}: {int(m.sum()):6d} instances, max {err[m].max():.2e}")
        worst = np.argsort(-err)[:8]
        lines.append("  worst: " + ", ".join(f"{int(i)} ({err[i]:.2e}, st {int(st[i])}, "
                                             f"{int(it[i])} it)" for i in worst))
        worst_all[name] = [[int(i), float(err[i]), int(st[i]), int(it[i])] for i in worst]
        np.savez(Path(report).parent / f"survey_worst_{name}.npz", idx=worst, err=err[worst],
                 U_gpu=_U[worst], U_opt=np.stack([res[i][3] for i in worst]))
        lines.append(f"  ({time.time() - t0:.0f} s)")
        print("\n".join(lines[first:]), flush=True)
    Path(report).parent.mkdir(parents=True, exist_ok=True)
    Path(report).write_text("\n".join(lines) + "\n")
    Path(report).with_suffix(".json").write_text(json.dumps(worst_all, indent=1))
    print("wrote", report)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("gpu", "cpu"))
    ap.add_argument("--sets", default=",".join(ALL))
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--report", default=str(REPO / "gpurun_out" / "parity_survey.txt"))
    ap.add_argument("--lib", default=None, help="gpu phase: a variant library")
    ap.add_argument("--param", action="append", default=[], help="gpu phase: SolverParams name=value")
    a = ap.parse_args()
    sets = [s for s in a.sets.split(",") if s]
    gpu(sets, a.lib, a.param) if a.mode == "gpu" else cpu(sets, a.procs, a.report)
