#!/bin/bash
# Product vs libpmc_codec_prev.so on one box at the three BASELINE sizes: the guard tests, then parity +
# A B A B at 10M x 1 KiB, 10M x 256 B and 1M x 4 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4ab3}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_fullsize.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T/k1 LIBS="libpmc_codec_prev.so libpmc_codec.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh || exit $?
TAG=$T/k4 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 4096 --n 1000000" bash scripts/gpu_variants.sh
