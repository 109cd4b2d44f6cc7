#!/bin/bash
# The whole -m gpu suite and smoke() on the current tree, then the default bench line.  Stops at the
# first failure.
#   TAG=r6suite bash scripts/gpu_suite.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bench_line.py $O/bench.json default
