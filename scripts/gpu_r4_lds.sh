#!/bin/bash
# Round 4: large-value parity + 64 KiB bench (chain-step prefetch), the front's LDS cost by phase (stop
# build), then product vs the ds_read_b64 window loads (PMC_LDS_B64) on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4lds}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_large.txt 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest_large.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --n 40000 --vlen 65536 --steps 2 > gpurun_out/$T/b_65536.json 2> gpurun_out/$T/b_65536.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/$T/b_65536.json'));print('65536',d['value'],d['compress_gib_s'],d['decompress_gib_s'],d['mismatches'])"
TAG=$T/lds bash scripts/front_lds.sh || exit $?
TAG=$T LIBS="libpmc_codec.so libpmc_codec_b64.so" bash scripts/gpu_variants.sh
