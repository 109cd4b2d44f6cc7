#!/bin/bash
# LDS / issue utilisation of the codec kernels: the counters this GPU offers, then PMC passes over a
# compress + decompress of N values (scripts/kernel_pmc.sh), one counter group per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-ldspmc}
mkdir -p gpurun_out/$T
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/$T/avail.txt 2>&1
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/$T/avail.txt | sort -u | tr '\n' ' ' > gpurun_out/$T/sq_counters.txt
echo; head -c 3000 gpurun_out/$T/sq_counters.txt; echo
TAG=$T/p1 CTRS="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
    bash scripts/kernel_pmc.sh || exit $?
cat gpurun_out/$T/p1/run.log | tail -3
TAG=$T/p2 CTRS="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
    bash scripts/kernel_pmc.sh
