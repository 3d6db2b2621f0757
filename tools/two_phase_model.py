"""Model of the two-phase straggler schedule, on the per-instance
anatomy of the config-3 batch (tools/diag_counts.py with CMPC_DIAG_SAVE, a -DCMPC_DIAG_COUNTS
build: wave cycles per instance, and the cycles / factorizations at the end of each of its first
four failed polish sessions).

Every rank's contiguous shard (N = 1, 2, 4, 8) is played through a queue-drain model of the
persistent one-wave kernels: W workers (2,048 = two NC <= 128 waves on each of the 1,024 SIMDs)
take the instances in queue order (the heavier bins first, as the kernels drain them), each
for its measured wall cycles.  The model's N = 8 / N = 1 ratio is checked against the measured
shard rehearsal before anything else is read from it.

Two-phase: an instance that fails its k-th polish session is parked there (phase 1 pays its
cycles up to that point) and finished by a four-wave team (cmpc_team.hip) on a CU of its own,
at `speed` x its one-wave rate -- either after phase 1 drains ("sequential"), or by T team
workgroups running beside phase 1 from the moment it is parked ("concurrent", T x 4 waves taken
from phase 1's pool).
   usage: python tools/two_phase_model.py DIAG_cfg3.npz [--measured N1_MS N8_MS]"""
import argparse
import heapq
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "convex-mpc-unitree-go2_amd"))


def drain(costs, W):
    """Persistent workers pulling a queue in order: start times, makespan."""
    h = [(0.0, w) for w in range(W)]
    heapq.heapify(h)
    start = np.empty(len(costs))
    end = 0.0
    for i, c in enumerate(costs):
        t, w = heapq.heappop(h)
        start[i] = t
        heapq.heappush(h, (t + c, w))
        end = max(end, t + c)
    return start, end


def queue_order(nc):
    """The kernels' drain order: bins NC 160, 144 (first class), then 128, 96; index order inside."""
    key = np.select([nc > 160, nc > 144, nc > 128, nc > 96], [0, 1, 2, 3], 4)
    return np.lexsort((np.arange(len(nc)), key))


def shard_makespans(cyc, nc, N, W, park_t=None, speed=2.0, mode="none", T=0):
    out = []
    B = len(cyc)
    for r in range(N):
        lo, hi = r * B // N, (r + 1) * B // N
        c, n = cyc[lo:hi], nc[lo:hi]
        o = queue_order(n)
        c = c[o]
        if mode == "none":
            out.append(drain(c, W)[1])
            continue
        p = park_t[lo:hi][o]
        parked = p > 0
        c1 = np.where(parked, p, c)
        rem = np.where(parked, c - p, 0.0) / speed
        if mode == "sequential":
            s, end1 = drain(c1, W)
            # phase 2: teams (one per CU: W / 8 of them) on an otherwise idle device
            _, end2 = drain(np.sort(rem[parked])[::-1], max(1, W // 8)) if parked.any() else (None, 0.0)
            out.append(end1 + end2)
        else:  # concurrent: T teams (4 waves each) beside phase 1 from the start
            s, end1 = drain(c1, W - 4 * T)
            ready = (s + c1)[parked]
            h = [0.0] * max(T, 1)
            end2 = 0.0
            for t_ready, rr in sorted(zip(ready, rem[parked])):
                t0 = max(heapq.heappop(h), t_ready)
                heapq.heappush(h, t0 + rr)
                end2 = max(end2, t0 + rr)
            out.append(max(end1, end2))
    return max(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--measured", type=float, nargs=2, default=None,
                    help="measured N = 1 and N = 8 step (ms) of the same build")
    a = ap.parse_args()
    from cmpc import synth
    z = np.load(a.npz)
    cyc = z["cyc"].astype(np.float64)
    ft = z["fail_t"].astype(np.float64)
    b = synth.make_config(3)
    nc = 3 * (b["contact"] != 0).reshape(len(cyc), -1).sum(1)
    W = 2048
    base = {N: shard_makespans(cyc, nc, N, W) for N in (1, 2, 4, 8)}
    print("current schedule (model): makespan cycles " +
          "  ".join(f"N={N}: {base[N]:.3g}" for N in base) +
          f"  -> N=8 speed-up {base[1] / base[8]:.2f}x")
    if a.measured:
        print(f"measured: N=1 {a.measured[0]} ms, N=8 {a.measured[1]} ms -> "
              f"{a.measured[0] / a.measured[1]:.2f}x; model cycles per ms at N=1 "
              f"{base[1] / a.measured[0]:.3g}, at N=8 {base[8] / a.measured[1]:.3g}")
    nf = (ft > 0).sum(1)
    print(f"instances with >= 1 / 2 / 3 failed sessions: {(nf >= 1).sum()} / {(nf >= 2).sum()} / "
          f"{(nf >= 3).sum()} of {len(cyc)}; slowest instance {cyc.max():.3g} cycles "
          f"(index {int(cyc.argmax())}, failed sessions {int(nf[cyc.argmax()])})")
    for k in (1, 2):
        park = np.where(nf >= k, ft[:, k - 1], 0.0)
        for speed in (1.5, 2.0, 3.0):
            seq = {N: shard_makespans(cyc, nc, N, W, park, speed, "sequential") for N in (1, 8)}
            line = (f"park at failed session {k}, team speed {speed}x: sequential N=1 "
                    f"{seq[1] / base[1]:.3f}x of today, N=8 {seq[8] / base[8]:.3f}x "
                    f"(speed-up {seq[1] / seq[8]:.2f}x)")
            for T in (16, 64):
                con = {N: shard_makespans(cyc, nc, N, W, park, speed, "concurrent", T)
                       for N in (1, 8)}
                line += (f"; concurrent T={T}: N=1 {con[1] / base[1]:.3f}x, N=8 "
                         f"{con[8] / base[8]:.3f}x (speed-up {con[1] / con[8]:.2f}x)")
            print(line)


if __name__ == "__main__":
    main()
