#!/bin/bash
# Round 5: the front's per-phase LDS cost (bank conflicts) and instruction mix per value, stop build.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5front}
TAG=$T/lds timeout -k 10 600 bash scripts/front_lds.sh > gpurun_out/$T.lds.txt 2>&1 || { cat gpurun_out/$T.lds.txt; exit 1; }
cat gpurun_out/$T.lds.txt
TAG=$T/cost timeout -k 10 600 bash scripts/front_cost.sh > gpurun_out/$T.cost.txt 2>&1 || { cat gpurun_out/$T.cost.txt; exit 1; }
cat gpurun_out/$T.cost.txt
