#!/bin/bash
# Round 4 front candidates on one box: parity + bench for each build (scripts/gpu_variants.sh), then the
# stamps build's eval counts for the product front and the gap front (1 KiB JSON).
#   product  libpmc_codec.so           (make)
#   s10      libpmc_codec_alt.so       -DPMC_FRONT_S10=1
#   gap      libpmc_codec_gap.so       -DPMC_FRONT_GAP=3
#   s10gap   libpmc_codec_s10gap.so    both
#   mt       libpmc_codec_mt.so        -DPMC_SPLIT_MT=1 (match-only token slab)
#   tskip    libpmc_codec_tskip.so     -DPMC_TREES_SKIP=1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4front}
mkdir -p gpurun_out/$T
for L in libpmc_codec_stamps.so libpmc_codec_stamps_gap.so; do
  PMC_LIB=$L timeout -k 10 300 python -u scripts/stamps.py 1024:0:400000 256:0:400000 > gpurun_out/$T/stamps_$L.txt 2>&1 || exit $?
  echo "== $L"; head -30 gpurun_out/$T/stamps_$L.txt
done
TAG=$T LIBS="${LIBS:-libpmc_codec.so libpmc_codec_alt.so libpmc_codec_gap.so libpmc_codec_mt.so}" bash scripts/gpu_variants.sh || exit $?
# LDS utilisation of the product front (bank conflicts vs LDS-active cycles)
TAG=$T/lds N=400000 CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
    bash scripts/kernel_pmc.sh
