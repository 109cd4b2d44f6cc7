#!/bin/bash
# Per-phase LDS cost of deflate_front_kernel (stop build, as scripts/front_cost.sh): LDS instructions,
# LDS-array cycles and bank-conflict cycles per value, by differences between consecutive phase stops.
#   TAG=x N=200000 [LIB=libpmc_codec_stop.so] bash scripts/front_lds.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PMC_LIB=${LIB:-libpmc_codec_stop.so}
OUT=gpurun_out/${TAG:-flds}
mkdir -p "$OUT"
N=${N:-200000}; V=${V:-1024}; K=${KIND:-0}
for st in 11 12 13 14 -1; do
    PMC_STOP_AFTER=$st timeout -k 10 300 rocprofv3 --kernel-trace \
        --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
        -d "$OUT/s$st" -o run --output-format csv -- python3 scripts/phase_drive.py $N $V $K > "$OUT/s$st.log" 2>&1 || exit $?
done
python3 - "$OUT" "$N" <<'PY'
import csv, os, sys
d, n = sys.argv[1], int(sys.argv[2])
keys = ["SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"]
prev = None
print(f"{'front phase (per value)':24s}" + "".join(f"{k[3:][:14]:>16s}" for k in keys))
for st, name in ((11, "stage"), (12, "sort"), (13, "chain counts"), (14, "parse+eval"), (-1, "histogram+out")):
    t = {}
    for r in csv.DictReader(open(os.path.join(d, f"s{st}", "run_counter_collection.csv"))):
        if "deflate_front_kernel" in r["Kernel_Name"]:
            t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cur = [t.get(k, 0.0) / n for k in keys]
    diff = cur if prev is None else [a - b for a, b in zip(cur, prev)]
    print(f"{name:24s}" + "".join(f"{v:16,.0f}" for v in diff))
    prev = cur
PY
