#!/bin/bash
# PMC counter passes over a 1M-value bench run (one rocprofv3 --pmc pass per counter group,
# kernel-trace only -- no system/runtime tracing beside counters), then the traffic summary.
#   TAG=... N=1000000 bash scripts/pmc_profile.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-pmc}
N=${N:-1000000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BENCH="bench.py --n $N --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
pass() {
    local name=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
        -- python3 $BENCH > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
pass mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES &&
pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE
rc=$?
find "$OUT" -name "*counter_collection.csv" | head -20
exit $rc
