#!/bin/bash
# Round 4: PMC_FRONT_PF (L2 prefetch of the next value) against the product, A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4pf} LIBS="libpmc_codec.so libpmc_codec_pf.so" bash scripts/gpu_variants.sh
