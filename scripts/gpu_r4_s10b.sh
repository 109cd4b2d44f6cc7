#!/bin/bash
# Round 4: PMC_FRONT_S10 (32 waves/CU) on top of the segmented eval maximum and the inlined front, A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4s10b} LIBS="libpmc_codec.so libpmc_codec_alt.so" bash scripts/gpu_variants.sh
