"""Summarise gpurun_out/<tag>/s*/run_counter_collection.csv into per-phase instruction
counts per value (deflate_small_kernel only)."""
import csv
import os
import sys

NAMES = {1: "stage+crc", 2: "sort", 3: "match_all", 4: "parse", 5: "histogram", 6: "lit+dist trees",
         7: "runs+bl tree+choice", 8: "emit", -1: "trailer+copy"}


def load(d):
    tot = {}
    f = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if "deflate_small_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def main(root, n):
    prev = None
    keys = ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"]
    print(f"{'phase':22s}" + "".join(f"{k[8:]:>14s}" for k in keys))
    for st in (1, 2, 3, 4, 5, 6, 7, 8, -1):
        d = os.path.join(root, f"s{st}")
        if not os.path.exists(d):
            continue
        t = load(d)
        row = {k: t.get(k, 0.0) - (prev.get(k, 0.0) if prev else 0.0) for k in keys}
        print(f"{NAMES[st]:22s}" + "".join(f"{row[k] / n:14,.0f}" for k in keys))
        prev = t
    print(f"{'TOTAL':22s}" + "".join(f"{prev.get(k, 0.0) / n:14,.0f}" for k in keys))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 200000)
