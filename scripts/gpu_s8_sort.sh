#!/bin/bash
# LDS atomic lane-order probe, then (if lanes get their old values in lane order) parity + A/B of
# the atomic-rank radix sort (B = libpmc_codec_alt.so built with -DPMC_SORT_ATOMIC_RANK).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_sort}
mkdir -p gpurun_out/$T
timeout -k 10 120 ./scripts/micro/lds_atomic_order > gpurun_out/$T/order.txt 2>&1; rc=$?
cat gpurun_out/$T/order.txt
[ $rc -eq 0 ] || exit $rc
TAG=$T/ab bash scripts/ab_check.sh
