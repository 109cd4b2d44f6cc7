#!/bin/bash
# Round 5 A/B libraries beside the product one (pmc_codec/lib*.so), from the working tree, for
# scripts/gpu_variants.sh (PMC_LIB selects one).  VARIANTS="name:flags ..." (default: the radix sort).
set -e
cd "$(dirname "$0")/.."
H="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden -Iinclude"
D=poor-man-s-cache_amd/pmc_codec
SRC=poor-man-s-cache_amd/csrc/pmc_codec.hip
make -s -C poor-man-s-cache_amd all > /dev/null
for v in ${VARIANTS:-radix:-DPMC_SORT_REG=0}; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc $H ${f//,/ } -o $D/libpmc_codec_$n.so $SRC &
done
wait
ls $D/*.so
