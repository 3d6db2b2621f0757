import sys, time, torch, numpy as np
sys.path.insert(0, 'convex-mpc-unitree-go2_amd')
from cmpc import Plan, SolverParams, to_device_batch, synth
B = 256
b = synth.make_batch(B, seed=1)
d = to_device_batch(b)
plan = Plan(SolverParams(max_batch=B))
w = torch.empty((B, 384), device='cuda'); st = torch.empty(B, dtype=torch.int32, device='cuda'); it = torch.empty_like(st)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it), stream=s)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
w_ref = w.clone()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it))
w.zero_()
g.replay(); torch.cuda.synchronize()
print("graph equal:", torch.equal(w, w_ref), st.min().item())
for name, fn in (("direct", lambda: plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it))), ("graph", g.replay)):
    for _ in range(5): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(50): fn()
    torch.cuda.synchronize(); print(name, (time.perf_counter() - t0) / 50 * 1e3, "ms")
# kernel time alone
plan.set_timing(True); plan.timing_read()
for _ in range(20): plan.solve(d["Ad"], d["Bd"], d["gd"], d["x0"], d["xref"], d["contact"], out=(w, st, it))
torch.cuda.synchronize(); ms, calls = plan.timing_read(); print("bin kernel ms/call", [m / max(c, 1) for m, c in zip(ms, calls)])
