#!/bin/bash
# Current-tree diagnostics: front stamps, per-phase front instruction counts, then every config.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_diag}
mkdir -p gpurun_out/$T
TAG=$T/stamps bash scripts/gpu_stamps.sh > /dev/null || exit $?
head -40 gpurun_out/$T/stamps.txt
TAG=$T/fcost bash scripts/front_cost.sh > gpurun_out/$T/front_cost.txt 2>&1 || exit $?
cat gpurun_out/$T/front_cost.txt
TAG=$T/cfg bash scripts/gpu_configs_r3.sh
