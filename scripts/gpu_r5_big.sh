#!/bin/bash
# Round 5: 30 KB values through the split pipeline's large pass (default) or the large-value pipeline
# (PMC_BIG_PASS=0), same box; then the large-value tests under PMC_BIG_PASS=0.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5big}
O=gpurun_out/$T
mkdir -p $O
for bp in 1 0 1 0; do
  PMC_BIG_PASS=$bp timeout -k 10 300 python bench.py --no-cpu-baseline --n 100000 --vlen 30000 --steps 2 > $O/b30k_$bp.json 2> $O/b30k_$bp.err || exit $?
  python3 scripts/bench_line.py $O/b30k_$bp.json "30K big_pass=$bp"
done
PMC_BIG_PASS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --n 500000 --vlen 20000 --steps 2 > $O/b20k_0.json 2> $O/b20k_0.err || exit $?
python3 scripts/bench_line.py $O/b20k_0.json "20K big_pass=0"
timeout -k 10 300 python bench.py --no-cpu-baseline --n 500000 --vlen 20000 --steps 2 > $O/b20k_1.json 2> $O/b20k_1.err || exit $?
python3 scripts/bench_line.py $O/b20k_1.json "20K big_pass=1"
PMC_BIG_PASS=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_codec.py -k "large or golden or ragged or multi_megabyte" > $O/pytest_bp0.txt 2>&1; rc=$?
tail -2 $O/pytest_bp0.txt; exit $rc
