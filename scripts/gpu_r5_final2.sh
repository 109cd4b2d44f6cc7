#!/bin/bash
# Round 5 final legs: every BASELINE config and the large values (scripts/gpu_configs_r5.sh), then the
# host/device batch table (bench --batches, host-ABI legs, host timers) and the single-value drop-in latency.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5cfg2}
O=gpurun_out/$T
mkdir -p $O
TAG=$T bash scripts/gpu_configs_r5.sh || exit $?
PMC_HOST_TRACE=1 timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
grep -v pmc_host_trace $O/batches.err | cut -c1-300
timeout -k 10 300 python scripts/latency_dropin.py --calls 500 > $O/latency_dropin.json 2> $O/latency_dropin.err || exit $?
cat $O/latency_dropin.err | tail -8
