#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/latk
for m in 0 1; do
  PMC_DEFLATE_MONO=$m timeout -k 10 120 python3 scripts/latency_kernels.py 1024 300 || exit $?
  PMC_DEFLATE_MONO=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/latk/m$m -o run -f csv -- python3 scripts/latency_kernels.py 1024 100 > /dev/null 2>&1 || exit $?
  head -12 gpurun_out/latk/m$m/run_kernel_stats.csv | cut -d, -f1-4
done
