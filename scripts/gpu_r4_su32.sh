#!/bin/bash
# Round 4: u32 sort counters (PMC_SORT_U32) and the segmented eval max (PMC_EVAL_SEGMAX) against the
# product: codec parity, the LDS phase
# attribution of both, A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4su32}
mkdir -p gpurun_out/$T
for L in su32 segmax; do
  PMC_LIB=libpmc_codec_$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_$L.txt 2>&1; rc=$?
  echo "$L: $(tail -1 gpurun_out/$T/pytest_$L.txt)"; [ $rc -eq 0 ] || exit $rc
done
TAG=$T/lds_su32 LIB=libpmc_codec_stop_su32.so bash scripts/front_lds.sh || exit $?
TAG=$T/k1 LIBS="libpmc_codec.so libpmc_codec_su32.so libpmc_codec_segmax.so" bash scripts/gpu_variants.sh
