#!/bin/bash
# Multi-block lane inflate pass (B = libpmc_codec_alt.so): coverage probe, parity suites, 64 KiB A/B, 1 MiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_mb}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_alt.so timeout -k 10 600 python3 scripts/inflate_probe.py 100000:128 300000:24 > gpurun_out/$T/probe.txt 2>&1; rc=$?
cat gpurun_out/$T/probe.txt; [ $rc -eq 0 ] || exit $rc
PMC_LIB=libpmc_codec_alt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_inflate_rec.py tests/test_gpu_alt_paths.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=$T/ab64k BENCH_ARGS="--n 40000 --vlen 65536 --steps 2" bash scripts/gpu_abab.sh || exit $?
PMC_LIB=libpmc_codec_alt.so timeout -k 10 400 python bench.py --no-cpu-baseline --n 1000 --vlen 1048576 --steps 1 > gpurun_out/$T/b1m.json 2> gpurun_out/$T/b1m.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/$T/b1m.json'));print('b1m',d['value'],d['compress_gib_s'],d['decompress_gib_s'],d['mismatches'],d['roofline']['kernel_ms_per_step'])"
