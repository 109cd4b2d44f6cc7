#!/bin/bash
# Round-3 closing GPU checks: the whole -m gpu suite, smoke(), then every config.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r3suite}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/smoke.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T/cfg bash scripts/gpu_configs_r3.sh || exit $?
OUT=gpurun_out/$T/refsrv timeout -k 10 900 bash scripts/ref_server_bench.sh > gpurun_out/$T/refsrv.log 2>&1; rc=$?
tail -6 gpurun_out/$T/refsrv.log; exit $rc
