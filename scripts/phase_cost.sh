#!/bin/bash
# Per-phase instruction counts of deflate_small_kernel: the stamps build ends every value
# after phase k (PMC_STOP_AFTER=k); differences of SQ counters between k and k-1 attribute
# instructions to phase k.  Phases: 1 stage+crc, 2 sort, 3 match_all, 4 parse,
# 5 histogram, 6 lit+dist trees, 7 runs+bl tree+block choice, 8 emit, -1 all.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PMC_LIB=libpmc_codec_stamps.so
OUT=gpurun_out/${TAG:-phase}
mkdir -p "$OUT"
N=${N:-200000}; V=${V:-1024}; K=${KIND:-0}
for st in 1 2 3 4 5 6 7 8 -1; do
    PMC_STOP_AFTER=$st timeout -k 10 300 rocprofv3 --kernel-trace \
        --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM \
        -d "$OUT/s$st" -o run --output-format csv -- python3 scripts/phase_drive.py $N $V $K > "$OUT/s$st.log" 2>&1 || exit $?
    echo "stop $st ok"
done
