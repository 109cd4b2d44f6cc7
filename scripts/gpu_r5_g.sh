#!/bin/bash
# Round 5: large-value routing for 16383..31808-byte values, the final-literal flush fix; large, codec,
# alternate-path and guard tests, the routing probe, then the 30 KB / 64 KiB legs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5g}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_alt_paths.py \
    tests/test_gpu_guard.py tests/test_gpu_codec.py tests/test_gpu_inflate_rec.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for cfg in "100000 30000" "40000 65536"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --n $1 --vlen $2 --steps 2 > $O/b_$2.json 2> $O/b_$2.err || exit $?
  python3 scripts/bench_line.py $O/b_$2.json "b_$2"
done
