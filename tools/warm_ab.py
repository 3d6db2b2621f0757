"""Diagnostic: throughput and per-bin kernel time of cold / warm solve variants on the bench's
next-tick scenario.  usage: python tools/warm_ab.py [config] [batch] [steps]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "convex-mpc-unitree-go2_amd")]
from cmpc import Plan, SolverParams, synth, to_device_batch  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
batch = synth.make_batch(B, seed=synth.CONFIGS[cfg]["seed"], mixed=synth.CONFIGS[cfg]["mixed"])
dev = torch.device("cuda", 0)
d = to_device_batch(batch, dev)
plan = Plan(SolverParams(max_batch=B))
y0 = torch.empty((B, 192), device=dev)
w0, _, _ = plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], y_out=y0)
g = torch.Generator(device=dev).manual_seed(1234)
sc = torch.tensor([2e-3] * 6 + [2e-2] * 6, device=dev)
d["x0"] = (d["x0"] + torch.randn(d["x0"].shape, generator=g, device=dev) * sc).contiguous()
y1 = torch.empty_like(y0)
w = torch.empty_like(w0)
st = torch.empty((B,), dtype=torch.int32, device=dev)
it = torch.empty_like(st)
variants = {
    "cold": {},
    "cold+y_out": dict(y_out=y1),
    "warm w": dict(w_init=w0),
    "warm y": dict(y_init=y0),
    "warm w,y": dict(w_init=w0, y_init=y0),
    "warm w,y+y_out": dict(w_init=w0, y_init=y0, y_out=y1),
}
for name, kw in variants.items():
    for _ in range(2):
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it), **kw)
    torch.cuda.synchronize()
    plan.timing_read()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(K):
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it), **kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    plan.set_timing(False)
    ms, calls = plan.timing_read()
    itn = it.cpu().numpy()
    print(f"{name:16s} {B * K / el / 1e6:6.3f} M/s  bins ms/step " +
          " ".join(f"{m / K:6.2f}" for m in ms) +
          f"  iters mean {itn.mean():.2f} max {itn.max()}  solved {(st == 1).float().mean().item():.4f}")
