#!/bin/bash
# Per-phase instruction counts of inflate_rec_kernel: the PMC_PHASE_STOP build ends the kernel's
# members after phase k (PMC_STOP_AFTER=31: prepare, 32: phase A, -1: all); differences of the SQ
# counters between passes attribute instructions to phases.  Per member; never quoted as timings.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PMC_LIB=libpmc_codec_stop.so
OUT=gpurun_out/${TAG:-reccost}
mkdir -p "$OUT"
N=${N:-200000}; V=${V:-1024}; K=${KIND:-0}
for st in 31 32 -1; do
    PMC_DRIVE_DECOMPRESS=1 PMC_STOP_AFTER=$st timeout -k 10 300 rocprofv3 --kernel-trace \
        --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM \
        -d "$OUT/s$st" -o run --output-format csv -- python3 scripts/phase_drive.py $N $V $K > "$OUT/s$st.log" 2>&1 || exit $?
    echo "stop $st ok"
done
python3 - "$OUT" "$N" <<'PY'
import csv, os, sys
d, n = sys.argv[1], int(sys.argv[2])
keys = ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"]
def tot(st):
    t = {}
    for r in csv.DictReader(open(os.path.join(d, f"s{st}", "run_counter_collection.csv"))):
        if "inflate_rec_kernel" in r["Kernel_Name"]:
            t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return t
prev = {k: 0.0 for k in keys}
print(f"{'phase (per member)':22s}" + "".join(f"{k[3:]:>14s}" for k in keys))
for st, name in ((31, "prepare"), (32, "phase A"), (-1, "phase B")):
    t = tot(st)
    print(f"{name:22s}" + "".join(f"{(t.get(k, 0) - prev[k]) / n:14,.0f}" for k in keys))
    prev = {k: t.get(k, 0.0) for k in keys}
PY
