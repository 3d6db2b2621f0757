"""Summarise rocprofv3 --pmc counter_collection.csv files for one kernel (diagnostic)."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    pat = sys.argv[2] if len(sys.argv) > 2 else "solve_bin_kernel<128>"
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat not in row.get("Kernel_Name", ""):
                    continue
                name = row["Counter_Name"]
                tot[name] += float(row["Counter_Value"])
                disp[name].add(row.get("Dispatch_Id", ""))
    for k in sorted(tot):
        n = max(len(disp[k]), 1)
        print(f"{k:32s} {tot[k] / n:16.4g}  (per dispatch, {n} dispatches)")
    w = tot.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in tot:
                print(f"  {k:28s} {100 * tot[k] / w:6.1f}% of wave cycles")


if __name__ == "__main__":
    main()
