"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches).
python scripts/pmc_summary.py gpurun_out/pmc"""
import csv
import os
import sys
from collections import defaultdict


def main(root):
    tot = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(set)
    for d in sorted(os.listdir(root)):
        f = os.path.join(root, d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k].add((d, r["Dispatch_Id"]))
    for k, c in tot.items():
        if "pmc" not in k:
            continue
        print(k)
        for n, v in sorted(c.items()):
            print(f"   {n:24s} {v:18,.0f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
