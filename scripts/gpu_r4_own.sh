#!/bin/bash
# Round 4: PMC_EVAL_OWNLOOP (eval owners by a scalar loop) against the product, with its codec parity first, A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_LIB=libpmc_codec_own.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_own.txt 2>&1; rc=$?
echo "own: $(tail -1 gpurun_out/pytest_own.txt)"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r4own} LIBS="libpmc_codec.so libpmc_codec_own.so" bash scripts/gpu_variants.sh
