#!/bin/bash
# lane_prepare / lane_block force-inlined again (the multi-block split had left them out of line):
# parity, A/B at 10M x 1 KiB and 40K x 64 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_inl}
mkdir -p gpurun_out/$T
TAG=$T/ab bash scripts/ab_check.sh || exit $?
TAG=$T/ab64k BENCH_ARGS="--n 40000 --vlen 65536 --steps 2" bash scripts/gpu_abab.sh
