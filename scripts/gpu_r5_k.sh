#!/bin/bash
# Round 5: 256 B / 4 KiB / alnum legs on the current tree (trees instance by size).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5k}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --vlen 256 > $O/b256.json 2> $O/b256.err || exit $?
python3 scripts/bench_line.py $O/b256.json b256
timeout -k 10 300 python bench.py --no-cpu-baseline --n 1000000 --vlen 4096 > $O/b4k.json 2> $O/b4k.err || exit $?
python3 scripts/bench_line.py $O/b4k.json b4k
