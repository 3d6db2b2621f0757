"""Diagnostic: per-instance cost anatomy (libcmpc_diag.so, -DCMPC_DIAG_COUNTS): iterations,
polish attempts, factorizations and wave cycles per instance; how much of the batch's wave time
the slowest instances take."""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def _lpt(cyc, W):
    import heapq
    h = [0.0] * W
    for cv in np.sort(cyc)[::-1]:
        heapq.heappush(h, heapq.heappop(h) + cv)
    return max(h)


def main():
    import torch
    from cmpc import _lib
    _lib._lib = _lib.load(os.environ.get("CMPC_DIAG_LIB", str(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_diag.so")))
    from cmpc import Plan, SolverParams, to_device_batch, synth
    over = dict(a.split("=") for a in sys.argv[1:])
    over = {k: type(getattr(SolverParams, k))(float(v) if "." in v else int(v)) for k, v in over.items()}
    plan = Plan(SolverParams(max_batch=65536, **over))
    for cfg in (1, 2, 3):
        b = synth.make_config(3) if cfg == 3 else synth.make_batch(65536, seed=cfg, mixed=cfg == 2)
        d = to_device_batch(b)
        w, st, it = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"])
        torch.cuda.synchronize()
        cyc = st.cpu().numpy().astype(np.float64) * 16
        code = it.cpu().numpy().astype(np.int64)
        iters, polraw, fac = code % 1000, (code // 1000) % 1000, code // 1000000
        # (+100 x flags: 1 loose acceptance, 2 certified face bound missed, 4 accepted on a
        # stalled downdated refinement -- cmpc_wave.hip solve_instance)
        flags, pol = polraw // 100, polraw % 100
        loose = flags & 1
        if os.environ.get("CMPC_DIAG_SAVE"):
            wh = w[:, :8].cpu().numpy()  # (diag build: cycles / factorizations at failed sessions 1..4)
            np.savez_compressed(f"{os.environ['CMPC_DIAG_SAVE']}_cfg{cfg}.npz", cyc=cyc, code=code,
                                fail_t=wh[:, :4], fail_f=wh[:, 4:8])
        order = np.argsort(-cyc)
        tot = cyc.sum()
        print(f"cfg{cfg} {over}: mean cycles {cyc.mean():.0f}  iters mean {iters.mean():.2f}  "
              f"polish {pol.mean():.2f}  fact {fac.mean():.2f}  loose acceptances "
              f"{int((loose > 0).sum())} of {len(cyc)}; certified bound missed "
              f"{int(((flags & 2) > 0).sum())}, stalled downdated refinement "
              f"{int(((flags & 4) > 0).sum())}")
        for frac in (0.001, 0.01, 0.05):
            k = max(1, int(frac * len(cyc)))
            top = order[:k]
            print(f"  top {frac*100:.1f}%: {100*cyc[top].sum()/tot:5.1f}% of cycles  iters {iters[top].mean():.1f}  "
                  f"polish {pol[top].mean():.1f}  fact {fac[top].mean():.1f}  cycles {cyc[top].mean():.0f}")
        print("  slowest instances:", order[:8].tolist(), "iters", iters[order[:8]].tolist(),
              "fact", fac[order[:8]].tolist())
        print(f"  max: cycles {cyc.max():.0f} iters {iters[order[0]]} polish {pol[order[0]]} fact {fac[order[0]]}")
        for q in (50, 90, 99, 99.9):
            print(f"  p{q}: cycles {np.percentile(cyc, q):.0f} iters {np.percentile(iters, q):.0f} fact {np.percentile(fac, q):.0f}")
        if cfg == 3:  # strong scaling: the slowest instance of each rank's contiguous shard
            for R in (1, 2, 4, 8):
                sh = np.array_split(cyc, R)
                print(f"  {R} ranks: shard max instance {max(x.max() for x in sh):.0f} cycles, "
                      f"mean per shard {np.mean([x.sum() for x in sh]):.3g}")
            nc = np.array([int(v) for v in d["contact"].reshape(65536, -1).ne(0).sum(1).cpu()]) * 3
            for lo, hi in ((0, 96), (97, 128), (129, 144), (145, 160), (161, 192)):
                m = (nc >= lo) & (nc <= hi)
                if m.any():
                    print(f"  bin <= {hi}: {m.sum()} inst, mean cycles {cyc[m].mean():.0f}, "
                          f"p99 {np.percentile(cyc[m], 99):.0f}, max {cyc[m].max():.0f}")
        if cfg == 1:  # one bin: persistent waves pulling the queue in (about) index order
            import heapq
            W = 2048  # 8 waves per CU x 256 CUs (NC = 128)
            h = [0.0] * W
            for cv in cyc:
                heapq.heappush(h, heapq.heappop(h) + cv)
            ideal = cyc.sum() / W
            print(f"  queue drain model: makespan {max(h):.0f} vs even share {ideal:.0f} cycles "
                  f"-> tail {100 * (max(h) / ideal - 1):.1f} %; sorted hardest-first "
                  f"{100 * (_lpt(cyc, W) / ideal - 1):.1f} %")


if __name__ == "__main__":
    main()
