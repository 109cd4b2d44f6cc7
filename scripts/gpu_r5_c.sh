#!/bin/bash
# Round 5: register bitonic sort in the front -- parity (goldens, ragged, digests at scale, multi-chunk
# full-size prefixes, guards) on the product build, then same-box A B A B against the radix sort.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5c}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_guard.py \
    tests/test_gpu_codec.py -k "fullsize or guard or golden or ragged or digest or roundtrip or latency_path" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T LIBS="${LIBS:-libpmc_codec.so libpmc_codec_radix.so}" timeout -k 10 1200 bash scripts/gpu_variants.sh
