#!/bin/bash
# Round 5, first GPU pass: the new parity tests (reference vectors above 82 KB, latency-path batches), the
# retry-list change (guard / alt-path / large tests), host-batch phase traces, single-value latency, default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5a}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_guard.py \
    tests/test_gpu_alt_paths.py "tests/test_gpu_codec.py" -k "large or guard or alt or latency_path or multi_megabyte or host_batch or golden or ragged" \
    > $O/pytest.txt 2>&1; rc=$?
tail -5 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
PMC_HOST_TRACE=1 timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
grep -v pmc_host_trace $O/batches.err | cut -c1-300
timeout -k 10 300 python scripts/latency_dropin.py --calls 500 > $O/latency_dropin.json 2> $O/latency_dropin.err || exit $?
cat $O/latency_dropin.err
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-600 $O/bench.json
