#!/bin/bash
# Round artifacts for bench.py's roofline object: FETCH_SIZE, WRITE_SIZE and issue-counter passes
# (separate rocprofv3 --pmc runs, kernel trace only) over one step of the default workload, then
# profiles/$ROUND/traffic.json (stamped with the library's source_id).  Stops on the first failure.
#   ROUND=r02 TAG=... bash scripts/round_pmc.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r02}
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" "profiles/$ROUND"
BENCH="bench.py --steps 1 --warmup 0 --no-cpu-baseline"
pass() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
        -- python3 $BENCH > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass issue SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE &&
python3 scripts/pmc_traffic.py "$OUT/fetch" "$OUT/write" 10000000 1024 0 "$OUT/issue" > "profiles/$ROUND/traffic.json"
rc=$?
echo "traffic rc=$rc"
cp "profiles/$ROUND/traffic.json" "$OUT/traffic.json" 2>/dev/null
exit $rc
