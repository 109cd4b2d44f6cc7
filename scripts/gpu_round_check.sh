#!/bin/bash
# One GPU call for a candidate tree: the whole -m gpu suite and smoke() (scripts/gpu_suite.sh, which ends
# with the default bench line), then same-box A B A B benches of LIBS with BENCH_ARGS (scripts/gpu_variants.sh).
#   TAG=x LIBS="libpmc_codec.so libpmc_codec_alt.so" BENCH_ARGS="--n 1000000 --vlen 4096" bash scripts/gpu_round_check.sh
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-check}
TAG=$TAG/suite bash scripts/gpu_suite.sh || exit $?
[ -n "${LIBS:-}" ] || exit 0
TAG=$TAG/ab bash scripts/gpu_variants.sh
