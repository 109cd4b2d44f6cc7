#!/bin/bash
# Round artifacts (one GPU call): PMC traffic/issue passes -> profiles/$ROUND/traffic.json (stamped with
# the kernel sources), the kernel-trace stats of the default bench command, then the plain default bench
# (which quotes the traffic file).  Stops at the first failure.
#   ROUND=r02 TAG=r2final bash scripts/round_artifacts.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r02}
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROUND=$ROUND TAG=$TAG bash scripts/round_pmc.sh > "$OUT/pmc.log" 2>&1 || { cat "$OUT/pmc.log"; exit 1; }
cat "$OUT/pmc.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- python3 bench.py --no-cpu-baseline \
    > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
rc=$?; echo "traced bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
exit $rc
