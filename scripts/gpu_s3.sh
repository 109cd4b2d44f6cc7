#!/bin/bash
# Candidate A/B (parity + A B A B), then the candidate's stamps diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s3}
mkdir -p gpurun_out/$T
TAG=$T/ab bash scripts/ab_check.sh || exit $?
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 300 python -u scripts/stamps.py > gpurun_out/$T/stamps.txt 2>&1; rc=$?
head -40 gpurun_out/$T/stamps.txt
exit $rc
