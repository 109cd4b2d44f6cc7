#!/bin/bash
# Eval stamps of a candidate stamps build (STAMPS_LIB, 1 KiB JSON slices), then scripts/gpu_variants.sh.
#   TAG=x STAMPS_LIB=libpmc_codec_k2stamps.so LIBS="libpmc_codec.so libpmc_codec_k2.so" bash scripts/gpu_variants_stamps.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-variants}
for S in ${STAMPS_LIB:-}; do
  PMC_LIB=$S timeout -k 10 240 python -u scripts/stamps.py ${STAMPS_CASES:-1024:0:400000} \
      > gpurun_out/${TAG:-variants}/stamps_$S.txt 2>&1 || exit $?
  grep -E "total|#evaluated|#consumed|#groups|parse |eval " gpurun_out/${TAG:-variants}/stamps_$S.txt | head -8
done
bash scripts/gpu_variants.sh
