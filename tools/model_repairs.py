"""Study (NumPy model, tests/algo_spec.py): what the polish repairs cost on config 3, and what
handling them without a factorization would save.  Runs the model on the slowest config-3
instances of the GPU diagnostics (profiles/r04d_diag_counts.txt) and on a random sample, with

  base         round 4's first kernel: face-adding repairs as downdates, 6 faces per factorization
  rebase       + a repair that drops only faces added by downdates re-downdates from the base
  weak         + faces ADMM holds weakly (gone at 40 % of its dual) enter as downdates
  ideal 5      every repair within 5 changed faces of the session's base costs no factorization
               and converges as a fresh one (an upper bound)
  border       the kernel's bordered repairs (cmpc_wave.hip border_build / border_apply: new
               parameters for dropped base faces, constraints for added ones, <= 5 columns, up to
               16 refinement steps on a border)
  border+r1    + one iterative-refinement step of every column W_j = M0 U_j

and prices each run with the measured per-phase costs of the light class (profiles/r04e_stamps:
131 k cycles per factorization, 12.6 k per refinement, 13 k per ADMM iteration, 11 k per face
downdate, 6.7 k per symv and 5.9 k per gradient in a border's columns).
    python tools/model_repairs.py [--sample 3000]
"""
import argparse
import sys
from multiprocessing import Pool
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))

import algo_spec  # noqa: E402
from cmpc import synth  # noqa: E402

SLOW = [52007, 30865, 28891, 25937, 14413, 795]
VARIANTS = [("base", dict(downdate=True, dd_max=6)),
            ("rebase", dict(downdate=True, dd_max=6, dd_rebase=True)),
            ("weak", dict(downdate=True, dd_max=6, dd_rebase=True, weak_base=0.6)),
            ("ideal 5", dict(downdate=True, dd_max=6, border_max=5)),
            ("border", dict(border=5, border_extra=12)),
            ("border+r1", dict(border=5, border_extra=12, border_refine=1))]
_B = None


def _run(i):
    inst = {k: _B[k][i] for k in ("Ad", "Bd", "gd", "x0", "xref", "contact")}
    out = []
    for n, kw in VARIANTS:
        o = algo_spec.solve(inst, algo_spec.Params(fp32_polish=True, **kw))
        refine_w = 1 if n.endswith("r1") else 0
        # border build: a symv per column, a gradient per new parameter; each column refinement
        # adds a gradient and a symv per column
        cols, ext = o.get("bd_cols", 0), o.get("bd_ext", 0)
        bcost = cols * 6.7 + ext * 5.9 + refine_w * cols * 12.6
        out.append((o["status"], o["iters"], o["fact"], o["refine"], o.get("dd_faces", 0), bcost))
    return i, out


def cost(x):
    return x[2] * 131 + x[3] * 12.6 + x[1] * 13 + x[4] * 11 + x[5]


def main():
    global _B
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", type=int, default=3000)
    a = ap.parse_args()
    _B = synth.make_config(3, B=65536)
    ids = SLOW + list(np.random.default_rng(0).choice(65536, a.sample, replace=False))
    with Pool(8) as pool:
        res = pool.map(_run, ids, chunksize=8)
    print("slowest config-3 instances (iterations / factorizations / model k cycles):")
    for i, r in res[:len(SLOW)]:
        print(f"  {i:5d} " + "  ".join(f"{n}: {x[1]}/{x[2]}/{cost(x):.0f}" for (n, _), x in zip(VARIANTS, r)))
    C = np.array([[cost(x) for x in r] for _, r in res[len(SLOW):]])
    F = np.array([[x[2] for x in r] for _, r in res[len(SLOW):]])
    print(f"random sample of {a.sample}:")
    for j, (n, _) in enumerate(VARIANTS):
        print(f"  {n:10s} mean {C[:, j].mean():6.1f} k cycles ({100 * (C[:, j].mean() / C[:, 0].mean() - 1):+5.1f} %)"
              f"  p99.9 {np.quantile(C[:, j], 0.999):5.0f}  max {C[:, j].max():5.0f}"
              f"  factorizations mean {F[:, j].mean():.3f} max {F[:, j].max()}")
    print("every run status 1:", all(x[0] == 1 for _, r in res for x in r))


if __name__ == "__main__":
    main()
