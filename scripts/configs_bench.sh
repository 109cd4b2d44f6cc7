#!/bin/bash
# The other BASELINE configurations (parity cases, not the headline line), one GPU call:
# 10M x 256 B, 1M x 4 KiB, 100K x 30 KB JSON slices, 1M x 1 KiB alnum, the SET/GET mix over the device
# slab, and the host-to-host (pinned, pipelined) leg of the headline workload.  Stops at the first failure.
#   TAG=cfg bash scripts/configs_bench.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfg}
mkdir -p "$OUT"
run() {
    local name=$1; shift
    timeout -k 10 600 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(round(d['value'],3), d['unit'], {k: round(v,3) for k, v in d.items() if k.endswith('_gib_s') or k in ('mops', 'ops_per_s')})" 2>/dev/null)"
    return $rc
}
run b256 --vlen 256 &&
run b4k --vlen 4096 --n 1000000 &&
run b30k --vlen 30000 --n 100000 &&
run alnum --kind 1 --n 1000000 &&
run mix --mix &&
run h2h --h2h
