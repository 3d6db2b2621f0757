"""Diagnostic: list instances whose status != 1 for a config/batch (writes JSON)."""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def main():
    from cmpc import Plan, SolverParams, solve_batch, synth
    out = {}
    plan = Plan(SolverParams(max_batch=65536))
    for cfg, B in ((1, 65536), (2, 65536), (3, 65536)):
        b = synth.make_config(cfg, B=B) if cfg == 3 else synth.make_batch(B, seed=synth.CONFIGS[cfg]["seed"], mixed=cfg == 2)
        w, st, it = solve_batch(b, plan=plan)
        bad = np.nonzero(st != 1)[0]
        out[f"cfg{cfg}"] = {"B": B, "bad": bad.tolist(), "status": st[bad].tolist(),
                            "iters": it[bad].tolist(), "iters_mean": float(it.mean()),
                            "iters_p99": float(np.percentile(it, 99)), "iters_max": int(it.max())}
        print(cfg, len(bad), out[f"cfg{cfg}"]["iters_mean"], out[f"cfg{cfg}"]["iters_p99"], flush=True)
    Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hard.json").write_text(json.dumps(out))


if __name__ == "__main__":
    main()
