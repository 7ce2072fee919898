"""Sum rocprofv3 --pmc CSV counters per kernel for one or more runs:
   python tools/pmc_summary.py <run_dir>... <kernel substring>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(run_dir, pat):
    tot = defaultdict(float)
    calls = set()
    for f in glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if pat in name:
                    tot[row["Counter_Name"]] += float(row["Counter_Value"])
                    calls.add(row.get("Dispatch_Id", ""))
    return tot, len(calls)


if __name__ == "__main__":
    *runs, pat = sys.argv[1:]
    for r in runs:
        tot, n = load(r, pat)
        print(f"{r}: {pat} dispatches={n} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items())))
