#!/bin/bash
# Back-kernel time when every value ends after phase k (stop build, PMC_STOP_AFTER=k: 21 stage,
# 22 crc, 23 codes, 24 tree headers, 25 symbols, -1 all), 2M x 1 KiB values, kernel trace only.  Diagnostic.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PMC_LIB=libpmc_codec_stop.so
OUT=gpurun_out/${TAG:-bstop}
mkdir -p "$OUT"
N=${N:-2000000}; V=${V:-1024}
for st in 21 22 23 24 25 -1; do
    PMC_STOP_AFTER=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/s$st" -o run -f csv \
        -- python3 scripts/phase_drive.py $N $V 0 > "$OUT/s$st.log" 2>&1 || exit $?
    python3 - "$OUT/s$st/run_kernel_stats.csv" $st <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "deflate_back_kernel" in r["Name"]:
        print("stop", sys.argv[2], "back ms", round(float(r["TotalDurationNs"]) / 1e6, 2), "launches", r["Calls"])
PY
done
