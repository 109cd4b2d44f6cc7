#!/bin/bash
# Round 4: the packed-S front (PMC_FRONT_S10, 32 waves/CU at <= 1 KiB) as build B (libpmc_codec_alt.so, built
# by hipcc -DPMC_FRONT_S10=1 from the working tree; A = `make`):
# parity on the codec suites, then a same-box A B A B bench at the headline config.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4s10}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_alt.so timeout -k 10 500 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_alt.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_alt.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T/ab bash scripts/gpu_abab.sh
