#!/bin/bash
# One PMC pass over a compress + decompress of N values: TAG=x CTRS="SQ_WAVES SQ_..." bash scripts/kernel_pmc.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kpmc}
mkdir -p "$OUT"
N=${N:-200000}; V=${V:-1024}; K=${KIND:-0}
PMC_DRIVE_DECOMPRESS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS \
    -d "$OUT" -o run --output-format csv -- python3 scripts/phase_drive.py $N $V $K > "$OUT/run.log" 2>&1 || exit $?
python3 - "$OUT" "$N" <<'PY'
import csv, os, sys
d, n = sys.argv[1], int(sys.argv[2])
tot = {}
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if not k.startswith("pmc::"):
        continue
    t = tot.setdefault(k, {})
    t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
keys = sorted({c for t in tot.values() for c in t})
print(f"{'kernel (per value)':34s}" + "".join(f"{k[3:][:13]:>14s}" for k in keys))
for k, t in sorted(tot.items()):
    print(f"{k[:34]:34s}" + "".join(f"{t.get(c, 0) / n:14,.0f}" for c in keys))
PY
