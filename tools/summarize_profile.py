"""Summarise one scripts/gpu_profile.sh run into profiles/ (kernel stats, HBM traffic, counters).

    python tools/summarize_profile.py --tag r02 [--root gpurun_out]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats of the headline run),
profiles/<tag>_kernel_trace_solve.csv (the solve-kernel rows of its trace: queue, start, end),
profiles/<tag>_hbm_traffic.json + profiles/hbm_traffic.json (PMC HBM bytes per launch of the
dominant kernel, the bench's ``roofline.traffic``), profiles/<tag>_counters.json +
profiles/counters.json (instruction-mix counters per launch: MFMA count, matrix-pipe
busy fraction, FP32 matrix TFLOP/s from the counted MFMAs), and copies the bench line.

Counter conventions (/opt/skills/guides/MI355X_MICROARCH.md): FETCH_SIZE / WRITE_SIZE in KB,
FETCH_SIZE doubled on gfx950 (wide reads are tallied at 64 B per 128-B request);
GRBM_GUI_ACTIVE sums the 8 XCDs (kernel GPU cycles = value / 8); SQ_VALU_MFMA_BUSY_CYCLES counts
busy cycles summed over SIMDs; one v_mfma_f32_16x16x4_f32 = 2 x 16 x 16 x 4 = 2,048 FLOP.
PMC runs serialise kernels, so per-dispatch counters are clean per kernel.
"""
import argparse
import csv
import glob
import json
import shutil
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SIMDS = 1024
MFMA_FLOP = 2048.0
PEAK_TFS = 157.3


def dispatches(root):
    """{(pass, dispatch_id): {"kernel": name, counter: value, ...}} over every PMC pass."""
    out = {}
    for f in glob.glob(f"{root}/pmc/p*/**/*counter_collection.csv", recursive=True):
        p = Path(f).relative_to(Path(root) / "pmc").parts[0]
        for r in csv.DictReader(open(f)):
            key = (p, r["Dispatch_Id"])
            d = out.setdefault(key, {"kernel": r["Kernel_Name"], "pass": p})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--root", default=str(REPO / "gpurun_out"))
    ap.add_argument("--side", action="store_true",
                    help="a side profile (not the headline): leave profiles/hbm_traffic.json and "
                         "profiles/counters.json alone")
    a = ap.parse_args()
    root = Path(a.root)
    out = REPO / "profiles"
    out.mkdir(exist_ok=True)
    stats = root / "prof" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, out / f"{a.tag}_kernel_stats.csv")
    trace = root / "prof" / "run_kernel_trace.csv"
    kern_ms = defaultdict(list)
    if trace.exists():
        rows = [r for r in csv.DictReader(open(trace)) if "solve_group_kernel" in r["Kernel_Name"]
                or "solve_team_kernel" in r["Kernel_Name"] or "bin_" in r["Kernel_Name"]]
        with open(out / f"{a.tag}_kernel_trace_solve.csv", "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Kernel_Name", "Queue_Id", "Start_Timestamp", "End_Timestamp", "Duration_ms"])
            for r in rows:
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                w.writerow([r["Kernel_Name"].split("(")[0], r["Queue_Id"], r["Start_Timestamp"],
                            r["End_Timestamp"], f"{dur:.4f}"])
                kern_ms[r["Kernel_Name"].split("(")[0]].append(dur)
    bench = root / "bench_full.json"
    if bench.exists():
        shutil.copy(bench, out / f"{a.tag}_bench.json")
    d = dispatches(root)
    per_kernel = defaultdict(lambda: defaultdict(list))
    for (p, _), r in d.items():
        if "solve_group_kernel" not in r["kernel"] and "solve_team_kernel" not in r["kernel"]:
            continue
        name = r["kernel"].split("(")[0]
        for k, v in r.items():
            if k not in ("kernel", "pass"):
                per_kernel[name][k].append(v)
    # every bench step of the headline is one full-batch launch per kernel: median launch
    summary = {}
    for name, cs in per_kernel.items():
        med = {k: sorted(v)[len(v) // 2] for k, v in cs.items()}
        s = {"launches": len(cs.get("FETCH_SIZE", cs.get("SQ_WAVES", []))), **med}
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            s["hbm_bytes_per_launch"] = (2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024.0
            s["hbm_bytes_per_launch_raw"] = (med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024.0
        if "SQ_INSTS_MFMA" in med and "GRBM_GUI_ACTIVE" in med:
            cyc = med["GRBM_GUI_ACTIVE"] / 8.0
            s["kernel_gpu_cycles"] = cyc
            s["mfma_busy_frac"] = med.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * SIMDS)
            s["mfma_flop_per_launch"] = med["SQ_INSTS_MFMA"] * MFMA_FLOP
            live = kern_ms.get(name)
            if live:
                ms = sorted(live)[len(live) // 2]
                s["trace_ms_median"] = ms
                s["mfma_tflops_at_trace_ms"] = med["SQ_INSTS_MFMA"] * MFMA_FLOP / (ms * 1e-3) / 1e12
                s["mfma_frac_of_peak"] = s["mfma_tflops_at_trace_ms"] / PEAK_TFS
        summary[name] = s
    (out / f"{a.tag}_counters.json").write_text(json.dumps(summary, indent=1))
    if not a.side:  # the bench's default --counters-json (the latest headline profile)
        (out / "counters.json").write_text(json.dumps(summary, indent=1))
    # dominant kernel (longest median trace duration) -> the bench's traffic figure
    dom = max(summary, key=lambda n: summary[n].get("trace_ms_median", 0.0)) if summary else None
    if dom and "hbm_bytes_per_launch" in summary[dom]:
        res = {"kernel": dom, "fetch_kb": summary[dom]["FETCH_SIZE"],
               "write_kb": summary[dom]["WRITE_SIZE"],
               "hbm_bytes_per_launch": summary[dom]["hbm_bytes_per_launch"],
               "hbm_bytes_per_launch_raw": summary[dom]["hbm_bytes_per_launch_raw"],
               "all_kernels": {n: s.get("hbm_bytes_per_launch") for n, s in summary.items()},
               "note": "per launch at the bench's headline batch (PMC, kernels serialised); fetch "
                       "doubled per the gfx950 FETCH_SIZE correction"}
        if not a.side:
            (out / "hbm_traffic.json").write_text(json.dumps(res, indent=1))
        (out / f"{a.tag}_hbm_traffic.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
