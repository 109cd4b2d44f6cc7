#!/bin/bash
# Round 5 closing run on the final sources: PMC traffic + kernel trace + default bench (round_artifacts.sh),
# then the whole -m gpu suite and smoke(), then every config leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5last}
O=gpurun_out/$T
mkdir -p $O
ROUND=r05 TAG=$T/art bash scripts/round_artifacts.sh > $O/art.log 2>&1 || { tail -20 $O/art.log; exit 1; }
tail -3 $O/art.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
TAG=$T/cfg bash scripts/gpu_configs_r5.sh || exit $?
timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
