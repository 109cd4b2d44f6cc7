#!/bin/bash
# Candidate libraries beside the product one (pmc_codec/libpmc_codec_<name>.so), built from the working
# tree with extra compile flags, for scripts/gpu_variants.sh / gpu_abab.sh (PMC_LIB selects one).  The
# product and fault builds come from `make`.
#   VARIANTS="alt:-DPMC_SOMETHING=1 other:-DX=2,-DY=3" bash scripts/build_variants.sh
set -e
cd "$(dirname "$0")/.."
H="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden -Iinclude"
D=poor-man-s-cache_amd/pmc_codec
SRC=poor-man-s-cache_amd/csrc/pmc_codec.hip
make -s -C poor-man-s-cache_amd all > /dev/null
for v in ${VARIANTS:?set VARIANTS=\"name:flags ...\"}; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc $H ${f//,/ } -o $D/libpmc_codec_$n.so $SRC &
done
wait
ls $D/*.so
