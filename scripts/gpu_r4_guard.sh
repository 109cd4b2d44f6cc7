#!/bin/bash
# Round 4: the lane-order guard tests, then the whole -m gpu suite and the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4guard}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_guard.txt 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_guard.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cat gpurun_out/$T/bench.json
