#!/bin/bash
# Round 4: sort and parse inlined into the front (PMC_FRONT_INLINE: no wave state in scratch) against the
# product: parity, per-value HBM bytes of both (FETCH_SIZE / WRITE_SIZE passes), A B A B at 1 KiB and 256 B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4inl}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_inl.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py tests/test_gpu_guard.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_inl.txt 2>&1; rc=$?
echo "inl: $(tail -1 gpurun_out/$T/pytest_inl.txt)"; [ $rc -eq 0 ] || exit $rc
for L in libpmc_codec.so libpmc_codec_inl.so; do
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== $L $C"; PMC_LIB=$L TAG=$T/pmc_${L}_$C N=400000 CTRS="$C" bash scripts/kernel_pmc.sh | grep "deflate_front\|kernel (per" || exit 1
  done
done
TAG=$T/k1 LIBS="libpmc_codec.so libpmc_codec_inl.so" bash scripts/gpu_variants.sh || exit $?
TAG=$T/b256 LIBS="libpmc_codec.so libpmc_codec_inl.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh
