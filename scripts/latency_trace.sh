#!/bin/bash
# Single-value latency breakdown: the drop-in latency script (untraced), then the same under a kernel +
# memory-copy trace (per-kernel and per-copy durations of one pmc_gzip_compress / _decompress call).
#   TAG=lat1 bash scripts/latency_trace.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lat}
mkdir -p "$OUT"
timeout -k 10 300 python3 scripts/latency_dropin.py --calls ${CALLS:-2000} > "$OUT/latency.json" 2> "$OUT/latency.err"
rc=$?; echo "latency rc=$rc"; cat "$OUT/latency.err"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace" -o run -f csv -- \
    python3 scripts/latency_dropin.py --calls 300 > "$OUT/latency_traced.json" 2> "$OUT/latency_traced.err"
rc=$?; echo "traced rc=$rc"
find "$OUT/trace" -name '*stats.csv' -exec sh -c 'echo "== $1"; head -30 "$1"' _ {} \;
exit $rc
