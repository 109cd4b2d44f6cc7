#!/bin/bash
# pmc_group host-to-host rates (1 and 2 contexts on the one GPU), then the LDS / issue PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s5}
mkdir -p gpurun_out/$T
timeout -k 10 400 python3 scripts/group_bench.py --n 1000000 > gpurun_out/$T/group.json 2> gpurun_out/$T/group.err || { tail -5 gpurun_out/$T/group.err; exit 1; }
cat gpurun_out/$T/group.err
TAG=$T/ldspmc bash scripts/gpu_lds_pmc.sh
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 300 python -u scripts/stamps.py 30000:0:20000 16000:0:20000 > gpurun_out/$T/stamps_big.txt 2>&1; cat gpurun_out/$T/stamps_big.txt
