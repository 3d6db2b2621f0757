"""How much faster a four-wave team (cmpc_team.hip) finishes the batch's slowest instances than
one wave does: each instance solved alone on the device (B = 1), in team mode (the one-per-CU
image) and in one-wave mode (cmpc_plan_set_team(0)), median of 5 launches each.  Input for the
two-phase straggler model (tools/two_phase_model.py `speed`).
   usage: python tools/straggler_speed.py DIAG_cfg3.npz [K]   (GPU)"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))
KEYS = ("Ad", "Bd", "gd", "x0", "xref", "contact")


def main():
    import torch
    from cmpc import Plan, SolverParams, to_device_batch, synth
    z = np.load(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    slow = np.argsort(-z["cyc"])[:k]
    b = synth.make_config(3)
    plan = Plan(SolverParams(max_batch=4))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ratios = []
    for i in slow:
        d = to_device_batch({kk: b[kk][i:i + 1] for kk in KEYS})
        res = {}
        for mode, team in (("team", -1), ("one-wave", 0)):
            plan.set_team(team)
            ms = []
            for _ in range(6):
                e0.record()
                w, st, it = plan.solve(*(d[kk] for kk in KEYS))
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            res[mode] = (float(np.median(ms[1:])), int(st.cpu()[0]), int(it.cpu()[0]))
        plan.set_team(-1)
        r = res["one-wave"][0] / res["team"][0]
        ratios.append(r)
        print(f"instance {int(i)}: in-batch {z['cyc'][i]:.3g} cycles; alone: team {res['team'][0]:.3f} ms "
              f"(status {res['team'][1]}, {res['team'][2]} it), one wave {res['one-wave'][0]:.3f} ms "
              f"(status {res['one-wave'][1]}, {res['one-wave'][2]} it) -> team {r:.2f}x", flush=True)
    print(f"team speed-up over one wave, alone: median {np.median(ratios):.2f}x, min {min(ratios):.2f}x")


if __name__ == "__main__":
    main()
