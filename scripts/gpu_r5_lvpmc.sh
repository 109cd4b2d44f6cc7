#!/bin/bash
# Round 5: HBM traffic and issue counters of the large-value kernels, 40K x 64 KiB (separate --pmc passes,
# kernel trace only), summarised per kernel by scripts/pmc_traffic.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5lvpmc}
O=gpurun_out/$T
mkdir -p $O
N=${N:-40000}; V=${V:-65536}
BENCH="bench.py --steps 1 --warmup 0 --no-cpu-baseline --n $N --vlen $V"
pass() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$O/$name" -o run --output-format csv \
        -- python3 $BENCH > "$O/$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass issue SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE &&
python3 scripts/pmc_traffic.py "$O/fetch" "$O/write" $N $V 0 "$O/issue" > "$O/traffic.json"
