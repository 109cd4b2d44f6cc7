#!/bin/bash
# Round 4 checkpoint: the whole -m gpu suite, smoke(), the default bench (with its CPU baseline), the
# kernel-trace summary of the default bench, then product vs PMC_TREES_SKIP at 10M x 256 B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4full}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.txt 2>&1 || exit $?
tail -2 gpurun_out/$T/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cat gpurun_out/$T/bench.json | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline > gpurun_out/$T/bench_traced.json 2> gpurun_out/$T/bench_traced.err || exit $?
TAG=$T/b256 LIBS="libpmc_codec.so libpmc_codec_tskip.so" BENCH_ARGS="--vlen 256" bash scripts/gpu_variants.sh
