#!/bin/bash
# Diagnostics of the working tree's kernels (one GPU call): the stamps build's per-phase cycle shares and
# event counts (scripts/stamps.py), then the front's per-phase instruction counts (scripts/front_cost.sh).
#   TAG=x bash scripts/gpu_diag.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-diag}
mkdir -p gpurun_out/$TAG
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 300 python -u scripts/stamps.py > gpurun_out/$TAG/stamps.txt 2>&1; rc=$?
cat gpurun_out/$TAG/stamps.txt
[ $rc -eq 0 ] || exit $rc
TAG=$TAG/fcost bash scripts/front_cost.sh > gpurun_out/$TAG/front_cost.txt 2>&1; rc=$?
cat gpurun_out/$TAG/front_cost.txt
exit $rc
