#!/bin/bash
# Per-phase instruction counts of deflate_back_kernel: the stop build ends every value after
# phase k (PMC_STOP_AFTER=k: 21 stage, 22 crc, 23 codes, 24 tree headers, 25 symbols, -1 all); differences
# of SQ counters between consecutive stops attribute instructions to a phase.
#   TAG=x N=200000 bash scripts/back_cost.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PMC_LIB=libpmc_codec_stop.so
OUT=gpurun_out/${TAG:-fcost}
mkdir -p "$OUT"
N=${N:-200000}; V=${V:-1024}; K=${KIND:-0}
for st in 21 22 23 24 25 -1; do
    PMC_STOP_AFTER=$st timeout -k 10 300 rocprofv3 --kernel-trace \
        --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM \
        -d "$OUT/s$st" -o run --output-format csv -- python3 scripts/phase_drive.py $N $V $K > "$OUT/s$st.log" 2>&1 || exit $?
done
python3 - "$OUT" "$N" <<'PY'
import csv, os, sys
d, n = sys.argv[1], int(sys.argv[2])
keys = ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"]
prev = None
print(f"{'front phase (per value)':24s}" + "".join(f"{k[3:]:>14s}" for k in keys))
for st, name in ((21, "stage"), (22, "crc"), (23, "codes"), (24, "runs+header"), (25, "symbols"), (-1, "trailer+copy")):
    t = {}
    for r in csv.DictReader(open(os.path.join(d, f"s{st}", "run_counter_collection.csv"))):
        if "deflate_back_kernel" in r["Kernel_Name"]:
            t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cur = [t.get(k, 0.0) / n for k in keys]
    diff = cur if prev is None else [a - b for a, b in zip(cur, prev)]
    print(f"{name:24s}" + "".join(f"{v:14,.0f}" for v in diff))
    prev = cur
PY
