"""Summarise rocprofv3 outputs of one bench run into profiles/ (kernel stats + HBM traffic).

    python tools/summarize_profile.py --tag r01 --stats gpurun_out/prof/run_kernel_stats.csv \
        --trace gpurun_out/prof/run_kernel_trace.csv --fetch gpurun_out/pmc_f/run_counter_collection.csv \
        --write gpurun_out/pmc_w/run_counter_collection.csv --batch 65536
"""
import argparse
import csv
import json
import shutil
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def per_dispatch(path, counter):
    vals = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = r["Dispatch_Id"]
        vals[d] += float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--kernel", default="solve_bin_kernel<128>")
    ap.add_argument("--bench")
    a = ap.parse_args()
    out = REPO / "profiles"
    out.mkdir(exist_ok=True)
    if a.stats:
        shutil.copy(a.stats, out / f"{a.tag}_kernel_stats.csv")
    if a.bench:
        shutil.copy(a.bench, out / f"{a.tag}_bench.json")
    res = {"kernel": a.kernel}
    if a.fetch and a.write:
        f, fm = per_dispatch(a.fetch, "FETCH_SIZE")
        w, wm = per_dispatch(a.write, "WRITE_SIZE")
        # the big-batch launches of the dominant kernel: longest dispatches
        ds = [d for d, m in fm.items() if a.kernel in m[0]]
        ds.sort(key=lambda d: -fm[d][2])
        top = ds[: max(1, len(ds) // 4)]
        fk = sum(f[d] for d in top) / len(top)
        dw = [d for d, m in wm.items() if a.kernel in m[0]]
        dw.sort(key=lambda d: -wm[d][2])
        topw = dw[: max(1, len(dw) // 4)]
        wk = sum(w[d] for d in topw) / len(topw)
        # FETCH_SIZE / WRITE_SIZE are KB; gfx950 FETCH_SIZE counts 64 B per 128-B request on
        # wide reads (MI355X_MICROARCH.md HBM section): report both raw and x2-corrected fetch
        res.update(fetch_kb=fk, write_kb=wk,
                   hbm_bytes_per_launch=(2 * fk + wk) * 1024.0,
                   hbm_bytes_per_launch_raw=(fk + wk) * 1024.0,
                   note="per launch of the dominant kernel at the bench batch; fetch doubled per "
                        "the gfx950 FETCH_SIZE correction")
        (out / "hbm_traffic.json").write_text(json.dumps(res, indent=1))
        (out / f"{a.tag}_hbm_traffic.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
