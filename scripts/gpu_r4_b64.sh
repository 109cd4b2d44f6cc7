#!/bin/bash
# Round 4: PMC_LDS_B64 window loads on top of the segmented eval maximum, A B A B at 1 KiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4b64} LIBS="libpmc_codec.so libpmc_codec_b64.so" bash scripts/gpu_variants.sh
