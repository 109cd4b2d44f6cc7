#!/bin/bash
# Round 4: aggregated sort atomics (PMC_SORT_AGG) against the product: parity, LDS phase attribution of
# both (stop builds), A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4agg}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_agg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_agg.txt 2>&1; rc=$?
echo "agg: $(tail -1 gpurun_out/$T/pytest_agg.txt)"; [ $rc -eq 0 ] || exit $rc
TAG=$T/lds LIB=libpmc_codec_stop.so bash scripts/front_lds.sh || exit $?
TAG=$T/lds_agg LIB=libpmc_codec_stop_agg.so bash scripts/front_lds.sh || exit $?
TAG=$T/k1 LIBS="libpmc_codec.so libpmc_codec_agg.so" bash scripts/gpu_variants.sh
