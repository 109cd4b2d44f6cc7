#!/bin/bash
# HBM deflate kernel at 8 waves per CU: parity (codec suite, incl. 1-4 MiB values), A/B at 64 KiB, B at 1 MiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_hbm}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_alt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=$T/ab64k BENCH_ARGS="--n 40000 --vlen 65536 --steps 2" bash scripts/gpu_abab.sh || exit $?
PMC_LIB=libpmc_codec_alt.so timeout -k 10 400 python bench.py --no-cpu-baseline --n 1000 --vlen 1048576 --steps 1 > gpurun_out/$T/b1m.json 2> gpurun_out/$T/b1m.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/$T/b1m.json'));print('b1m',d['value'],d['compress_gib_s'],d['decompress_gib_s'],d['mismatches'],d['roofline']['kernel_ms_per_step'])"
