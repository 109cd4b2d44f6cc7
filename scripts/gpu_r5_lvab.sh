#!/bin/bash
# Round 5: same-box A/B of large-value parse variants (PMC_LIB): large-value parity per library, then the
# 64 KiB and 30 KB legs for each in turn, twice round.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5lvab}
O=gpurun_out/$T
mkdir -p $O
for L in $LIBS; do
  PMC_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 240 --timeout-method thread \
      > $O/pytest_$L.txt 2>&1; rc=$?
  echo "$L parity: $(tail -1 $O/pytest_$L.txt)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for L in $LIBS; do
    for cfg in "40000 65536" "100000 30000"; do
      set -- $cfg
      PMC_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --n $1 --vlen $2 --steps 2 > $O/b_${L}_$2_$r.json \
          2> $O/b_${L}_$2_$r.err || exit $?
      python3 scripts/bench_line.py $O/b_${L}_$2_$r.json "$L $2 r$r"
    done
  done
done
