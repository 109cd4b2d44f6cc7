#!/bin/bash
# Measurement of the front on the current tree:
# eval stamps (positions evaluated vs consumed, lanes, steps), per-phase instruction and LDS counters,
# then one default bench line.  Every GPU step has its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-front}
mkdir -p "$OUT"
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 240 python -u scripts/stamps.py 1024:0:400000 4096:0:100000 \
    > "$OUT/stamps.txt" 2>&1 || exit $?
TAG=${TAG:-front}/fcost N=200000 bash scripts/front_cost.sh > "$OUT/front_cost.txt" 2>&1 || exit $?
TAG=${TAG:-front}/flds N=200000 bash scripts/front_lds.sh > "$OUT/front_lds.txt" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -n 1 "$OUT/bench.json"
