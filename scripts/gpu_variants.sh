#!/bin/bash
# Same-box comparison of several builds of the codec library (pmc_codec/<lib>): golden parity for each,
# then the default bench for each in turn, twice round (box-to-box clock differences cancel).
#   TAG=x LIBS="libpmc_codec.so libpmc_codec_alt.so" bash scripts/gpu_variants.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-variants}
mkdir -p gpurun_out/$T
LIBS=${LIBS:-libpmc_codec.so libpmc_codec_alt.so}
for L in $LIBS; do
  PMC_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu -k "golden or ragged" --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_$L.txt 2>&1; rc=$?
  echo "$L parity: $(tail -1 gpurun_out/$T/pytest_$L.txt)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for L in $LIBS; do
    PMC_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$T/b_${L}_$r.json 2> gpurun_out/$T/b_${L}_$r.err || exit $?
    python3 - gpurun_out/$T/b_${L}_$r.json "$L r$r" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = d["roofline"]["kernel_ms_per_step"]
print(sys.argv[2], round(d["value"], 3), round(d["compress_gib_s"], 3), round(d["decompress_gib_s"], 3),
      d.get("fullsize_parity", {}).get("match"), {n.split("::")[1][:22]: round(v, 1) for n, v in ks.items() if v > 1})
PY
  done
done
