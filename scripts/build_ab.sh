#!/bin/bash
# Builds the two libraries of a same-box A/B (scripts/ab_check.sh, gpu_abab.sh), in this container:
#   A = pmc_codec/libpmc_codec.so      from the committed tree (git HEAD, or $BASE)
#   B = pmc_codec/libpmc_codec_alt.so  from the working tree
# (EXTRA_B="-DX=1" adds flags to B only.)  Run `make -C poor-man-s-cache_amd` afterwards to put the working tree's build back as A.
set -e
cd "$(dirname "$0")/.."
BASE=${BASE:-HEAD}
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden"
/opt/rocm/bin/hipcc $HIPFLAGS ${EXTRA_B:-} -Iinclude -o poor-man-s-cache_amd/pmc_codec/libpmc_codec_alt.so \
    poor-man-s-cache_amd/csrc/pmc_codec.hip &
T=$(mktemp -d)
git archive "$BASE" poor-man-s-cache_amd/csrc include | tar -x -C "$T"
/opt/rocm/bin/hipcc $HIPFLAGS -I"$T/include" -o poor-man-s-cache_amd/pmc_codec/libpmc_codec.so \
    "$T/poor-man-s-cache_amd/csrc/pmc_codec.hip"
wait
rm -rf "$T"
# A is a HEAD build with a fresh mtime: make the working-tree sources newer so the next `make` rebuilds it
touch poor-man-s-cache_amd/csrc/pmc_codec.hip
echo "A = $BASE, B = working tree"
