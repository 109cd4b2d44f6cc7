#!/bin/bash
# kernel-trace stats of a reduced bench run: TAG=x N=1000000 bash scripts/gpu_ktrace.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-kt}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run -f csv -- python3 bench.py --n ${N:-1000000} --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "traced bench rc=$rc"; cat "$OUT/bench.json" | cut -c1-300
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} total_ms {float(r['TotalDurationNs'])/1e6:10.2f} avg_us {float(r['AverageNs'])/1e3:10.1f}")
PY
exit $rc
