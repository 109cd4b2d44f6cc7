#!/bin/bash
# Round 4: canonical-code ranks by ballots in the back (PMC_CODES_BALLOT) against the product: parity,
# A B A B at 1 KiB and 256 B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4cb}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_cb.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_cb.txt 2>&1; rc=$?
echo "cb: $(tail -1 gpurun_out/$T/pytest_cb.txt)"; [ $rc -eq 0 ] || exit $rc
TAG=$T/k1 LIBS="libpmc_codec.so libpmc_codec_cb.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec.so libpmc_codec_cb.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh
