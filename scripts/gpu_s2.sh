#!/bin/bash
# Candidate A/B (parity + A B A B), drop-in latency of A and B, B's latency trace, then diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s2}
mkdir -p gpurun_out/$T
TAG=$T/ab bash scripts/ab_check.sh || exit $?
timeout -k 10 300 python3 scripts/latency_dropin.py --calls 1000 > gpurun_out/$T/latency_A.json 2> gpurun_out/$T/latency_A.err || exit $?
cat gpurun_out/$T/latency_A.err
PMC_LIB=libpmc_codec_alt.so timeout -k 10 300 python3 scripts/latency_dropin.py --calls 1000 > gpurun_out/$T/latency_B.json 2> gpurun_out/$T/latency_B.err || exit $?
cat gpurun_out/$T/latency_B.err
PMC_LIB=libpmc_codec_alt.so timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/$T/lat_trace -o run -f csv -- \
    python3 scripts/latency_dropin.py --calls 200 > gpurun_out/$T/lat_traced.json 2> gpurun_out/$T/lat_traced.err || exit $?
find gpurun_out/$T/lat_trace -name '*stats.csv' -exec sh -c 'echo "== $1"; head -25 "$1"' _ {} \;
TAG=$T/diag bash scripts/gpu_diag.sh
