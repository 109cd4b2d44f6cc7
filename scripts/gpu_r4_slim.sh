#!/bin/bash
# Round 4: the slimmed wave state + register-free code-rank guard (product) against the previous product
# build (libpmc_codec_prev.so), guard tests first; then the same pair at 256 B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4slim}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_guard.txt 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest_guard.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T/k1 LIBS="libpmc_codec_prev.so libpmc_codec.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh
