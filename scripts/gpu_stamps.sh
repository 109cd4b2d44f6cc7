#!/bin/bash
# Diagnostic: per-phase wave-cycle shares and event counts of the front (PMC_STAMPS build).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 300 python -u scripts/stamps.py > gpurun_out/${TAG:-stamps}.txt 2>&1; rc=$?
cat gpurun_out/${TAG:-stamps}.txt; exit $rc
