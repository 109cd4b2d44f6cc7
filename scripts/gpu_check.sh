#!/bin/bash
# GPU parity run: smoke() then pytest -m gpu.  Stops after a fault/abort/timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; tail -5 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -40 gpurun_out/pytest_gpu.log
exit $rc
