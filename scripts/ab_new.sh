#!/bin/bash
# Parity of the product build (codec, full-size and alternate-path GPU tests), then a same-box
# A B A B bench against PMC_LIB=$ALT (the previous formulation).
#   TAG=x ALT=libpmc_codec_alt.so bash scripts/ab_new.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-abn}
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py \
    tests/test_gpu_alt_paths.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ALT=${ALT:-libpmc_codec_alt.so} TAG=$TAG bash scripts/gpu_abab.sh
