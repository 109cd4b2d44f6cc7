#!/bin/bash
# One GPU call: the GPU suite + default bench on the product library (A), then the codec parity tests
# on the candidate build (PMC_LIB=$ALT) and a same-box A B A B bench.  Stops at the first failure.
#   TAG=x ALT=libpmc_codec_alt.so bash scripts/gpu_suite_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-sab}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json
[ $rc -eq 0 ] || exit $rc
TAG=$TAG/ab bash scripts/ab_check.sh
