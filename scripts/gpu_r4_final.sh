#!/bin/bash
# Round 4 artifacts from the final tree: the whole -m gpu suite, smoke(), the kernel-trace summary of the
# default bench, the PMC traffic passes (profiles/r04/traffic.json, stamped with the sources' id), the
# default bench with that roofline, the server-shaped batch leg and its kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit $?
ROUND=r04 TAG=$T/pmc timeout -k 10 600 bash scripts/round_pmc.sh > $O/round_pmc.log 2>&1 || { tail -5 $O/round_pmc.log; exit 1; }
tail -2 $O/round_pmc.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-400 $O/bench.json
timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_batches -o run --output-format csv \
    -- python3 bench.py --batches > $O/batches_traced.json 2> $O/batches_traced.err || exit $?
exit 0
