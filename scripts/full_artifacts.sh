#!/bin/bash
# Round artifacts: kernel-trace stats of the default bench command, PMC traffic passes,
# then the plain default bench (which picks up profiles/traffic.json).  Stops on failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- python3 bench.py --h2h \
    > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
rc=$?; echo "traced bench rc=$rc"; cat "$OUT/bench_traced.json"
if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$c" -o run -f csv -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$c.log" 2>&1
    rc=$?; echo "pmc $c rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
mkdir -p profiles
python3 scripts/pmc_traffic.py "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" 10000000 1024 0 > profiles/traffic.json
rc=$?; echo "traffic rc=$rc"; cat profiles/traffic.json
cp profiles/traffic.json "$OUT/traffic.json"
timeout -k 10 900 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
exit $rc
