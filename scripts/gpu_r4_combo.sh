#!/bin/bash
# Round 4 combined: aggregated sort atomics parity; LDS phase attribution of the product, PMC_SORT_AGG and
# PMC_LDS_B64 (stop builds); A B A B of prev / product / agg at 1 KiB, prev / product at 256 B and 4 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4combo}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_agg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_agg.txt 2>&1; rc=$?
echo "agg: $(tail -1 gpurun_out/$T/pytest_agg.txt)"; [ $rc -eq 0 ] || exit $rc
for L in stop stop_agg stop_b64; do
  echo "== $L"; TAG=$T/lds_$L LIB=libpmc_codec_$L.so N=100000 bash scripts/front_lds.sh || exit $?
done
TAG=$T/k1 LIBS="libpmc_codec_prev.so libpmc_codec.so libpmc_codec_agg.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh || exit $?
TAG=$T/k4 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 4096 --n 1000000" bash scripts/gpu_variants.sh
