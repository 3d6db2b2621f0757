"""Diagnostic: per-phase cycle shares of the solve kernel (libcmpc_stamps.so, -DCMPC_STAMPS).

    python tools/stamps.py [--config 1] [--batch 8192]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--lib", default=str(REPO / "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_stamps.so"))
    ap.add_argument("--warm", action="store_true",
                    help="measure the bench's next-tick warm-start scenario (cold twin first)")
    ap.add_argument("--team", type=int, default=-1, help="cmpc_plan_set_team (-1 auto, 0 off)")
    ap.add_argument("--only-bin", type=int, default=-1, help="keep only instances of this bin (0-4)")
    a = ap.parse_args()
    import torch
    from cmpc import _lib, synth
    lib = _lib.load(Path(a.lib))
    _lib._lib = lib
    lib.cmpc_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    from cmpc import Plan, SolverParams, to_device_batch
    b = synth.make_batch(a.batch, seed=1, mixed=(a.config == 2))
    if a.only_bin >= 0:
        nf = 3 * (b["contact"] != 0).reshape(a.batch, -1).sum(1)
        keep = np.searchsorted(np.array([96, 128, 144, 160, 192]), nf) == a.only_bin
        b = {k: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == keep.shape else v) for k, v in b.items()}
        a.batch = int(keep.sum())
        print("instances kept:", a.batch)
    d = to_device_batch(b)
    plan = Plan(SolverParams(max_batch=a.batch))
    plan.set_team(a.team)
    buf = (ctypes.c_ulonglong * 32)()
    kw = {}
    if a.warm:
        y0 = torch.empty((a.batch, 12 * 16), dtype=torch.float32, device=d["Ad"].device)
        w0, _, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], y_out=y0)
        g = torch.Generator(device=d["Ad"].device).manual_seed(1234)
        sc = torch.tensor([2e-3] * 6 + [2e-2] * 6, device=d["Ad"].device)
        d["x0"] = (d["x0"] + torch.randn(d["x0"].shape, generator=g, device=d["Ad"].device) * sc).contiguous()
        torch.cuda.synchronize()
        report(lib, plan, d, buf, {}, "cold (next tick)")
        kw = dict(w_init=w0, y_init=y0, y_out=torch.empty_like(y0))
    report(lib, plan, d, buf, kw, "warm (next tick)" if a.warm else "cold")


def report(lib, plan, d, buf, kw, title):
    import torch
    plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], **kw)
    torch.cuda.synchronize()
    lib.cmpc_debug_stamps(buf)
    r = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], **kw)
    st = r[1]
    torch.cuda.synchronize()
    lib.cmpc_debug_stamps(buf)
    v = np.array(list(buf), dtype=np.float64)
    n = v[10]
    names = ["condense", "invert", "gradient", "symv", "polish(all, incl. grad/symv)",
             "instance total", "setup", "admm rest", None, None, None, None, None, None,
             "polish setup", "output"]
    print(f"== {title}")
    print(f"instances {int(n)}  mean iters {v[11]/n:.2f}  condense_invert/inst {v[8]/n:.2f}  "
          f"polish attempts/inst {v[9]/n:.2f}")
    for i, nm in enumerate(names):
        if nm is None:
            continue
        print(f"  {nm:28s} {v[i]/n:12.0f} cycles/instance  {100*v[i]/v[5]:5.1f}%")
    print(f"  per call: condense {v[0]/v[8]:.0f}  invert {v[1]/v[8]:.0f}  gradient {v[2]/max(v[12],1):.0f} (x{v[12]/n:.1f})  symv {v[3]/max(v[13],1):.0f} (x{v[13]/n:.1f}) cycles")
    if v[29] > 0:
        print(f"  face downdates: {v[29]/n:.3f} repairs/instance ({v[30]/v[29]:.2f} faces each), "
              f"{v[28]/v[29]:.0f} cycles per repair, {100*v[28]/v[5]:.1f}% of the total")
    if v[16] + v[19] > 0:
        print(f"  team factor per call: backward {v[16]/v[8]:.0f}  forward {v[17]/v[8]:.0f}  "
              f"mirror+scale {v[18]/v[8]:.0f}  sweep {v[19]/v[8]:.0f} cycles")
        print(f"  team sweep per call: publish {v[20]/v[8]:.0f}  barrier {v[21]/v[8]:.0f}  "
              f"LDL+MFMA {v[22]/v[8]:.0f} cycles; helpers' barrier waits (sum) {v[23]/v[8]:.0f}")
    if v[25] > 0:
        print(f"  team symv per call: issue {v[24]/v[13]:.0f}  part {v[25]/v[13]:.0f}  "
              f"barrier {v[26]/v[13]:.0f}  reduce {v[27]/v[13]:.0f} cycles")
    print("  status:", dict(zip(*np.unique(st.cpu().numpy(), return_counts=True))))

if __name__ == "__main__":
    main()
