#!/bin/bash
# Round 5: small batches of 16-32 KB values back through the large pass -- codec, large, drop-in and
# alternate-path tests, then the single-value drop-in latency and the 30 KB leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5route}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_large.py \
    tests/test_gpu_alt_paths.py tests/test_kvs_dropin.py -m gpu > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/latency_dropin.py --calls 200 > $O/latency_dropin.json 2> $O/latency_dropin.err || exit $?
tail -2 $O/latency_dropin.err
timeout -k 10 300 python bench.py --no-cpu-baseline --n 100000 --vlen 30000 --steps 2 > $O/b30k.json 2> $O/b30k.err || exit $?
python3 scripts/bench_line.py $O/b30k.json b30k
