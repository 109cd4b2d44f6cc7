#!/bin/bash
# Builds the round's candidate libraries beside the product one (pmc_codec/lib*.so), from the working
# tree, for scripts/gpu_variants.sh / gpu_r4_front.sh (PMC_LIB selects one).  The product and fault
# builds come from `make`.
set -e
cd "$(dirname "$0")/.."
H="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden -Iinclude"
D=poor-man-s-cache_amd/pmc_codec
SRC=poor-man-s-cache_amd/csrc/pmc_codec.hip
make -C poor-man-s-cache_amd -j4 > /dev/null
b() { /opt/rocm/bin/hipcc $H "${@:2}" -o $D/$1 $SRC; }
b libpmc_codec_alt.so -DPMC_FRONT_S10=1 &
b libpmc_codec_gap.so -DPMC_FRONT_GAP=3 &
b libpmc_codec_s10gap.so -DPMC_FRONT_GAP=3 -DPMC_FRONT_S10=1 &
b libpmc_codec_mt.so -DPMC_SPLIT_MT=1 &
wait
b libpmc_codec_tskip.so -DPMC_TREES_SKIP=1 &
b libpmc_codec_b64.so -DPMC_LDS_B64=1 &
b libpmc_codec_stop.so -DPMC_PHASE_STOP &
b libpmc_codec_stamps.so -DPMC_STAMPS &
b libpmc_codec_stamps_gap.so -DPMC_STAMPS -DPMC_FRONT_GAP=3 &
wait
ls -la $D/*.so
