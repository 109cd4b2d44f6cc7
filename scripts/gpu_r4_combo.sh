#!/bin/bash
# Round 4 combined: aggregated sort atomics (PMC_SORT_AGG) and ballot-built HC (PMC_HC_BALLOT) parity; LDS phase attribution of the product, PMC_SORT_AGG and
# PMC_LDS_B64 (stop builds); A B A B of prev / product / agg at 1 KiB, prev / product at 256 B and 4 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4combo}
mkdir -p gpurun_out/$T
for V in agg hcb; do
  PMC_LIB=libpmc_codec_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_$V.txt 2>&1; rc=$?
  echo "$V: $(tail -1 gpurun_out/$T/pytest_$V.txt)"; [ $rc -eq 0 ] || exit $rc
done
for L in stop stop_agg stop_b64; do
  echo "== $L"; TAG=$T/lds_$L LIB=libpmc_codec_$L.so N=100000 bash scripts/front_lds.sh || exit $?
done
TAG=$T/k1 LIBS="libpmc_codec_prev.so libpmc_codec.so libpmc_codec_agg.so libpmc_codec_hcb.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh || exit $?
TAG=$T/k4 LIBS="libpmc_codec_prev.so libpmc_codec.so" BENCH_ARGS="--vlen 4096 --n 1000000" bash scripts/gpu_variants.sh
