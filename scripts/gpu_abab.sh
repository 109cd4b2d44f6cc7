#!/bin/bash
# Same-box A/B of two builds: bench with the product library (A) and PMC_LIB=$ALT (B),
# alternating A B A B so box-to-box clock differences cancel.
#   TAG=x ALT=libpmc_codec_alt.so bash scripts/gpu_abab.sh
# (ENV_B="VAR=value ..." sets B's environment, e.g. ALT=libpmc_codec.so ENV_B=PMC_INFLATE_REC=0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-abab}
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_A$r.json 2> gpurun_out/${TAG}_A$r.err || exit $?
  env ${ENV_B:-} PMC_LIB=${ALT:-libpmc_codec_alt.so} timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_B$r.json 2> gpurun_out/${TAG}_B$r.err || exit $?
done
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for k in ("A1", "B1", "A2", "B2"):
    d = json.load(open(f"gpurun_out/{t}_{k}.json"))
    ks = d["roofline"]["kernel_ms_per_step"]
    print(k, round(d["value"], 3), round(d["compress_gib_s"], 3), round(d["decompress_gib_s"], 3),
          {n.split("::")[1][:22]: round(v, 1) for n, v in ks.items() if v > 1})
PY
