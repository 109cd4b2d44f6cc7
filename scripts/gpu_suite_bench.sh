#!/bin/bash
# GPU suite, then the default bench (driver-shaped), into gpurun_out/$TAG.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-suite}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cat gpurun_out/$T/bench.json
