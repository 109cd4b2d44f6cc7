#!/bin/bash
# Trees kernel with the lengths row staged in LDS: parity, A/B at 1 KiB and 256 B, lone-value latency.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_trees}
mkdir -p gpurun_out/$T
TAG=$T/ab bash scripts/ab_check.sh || exit $?
TAG=$T/ab256 BENCH_ARGS="--vlen 256" bash scripts/gpu_abab.sh || exit $?
PMC_LIB=libpmc_codec_alt.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/lat -o run -f csv -- python3 scripts/latency_kernels.py 1024 100 > /dev/null 2>&1 || exit $?
head -5 gpurun_out/$T/lat/run_kernel_stats.csv | cut -d, -f1-4
