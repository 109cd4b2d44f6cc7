#!/bin/bash
# Round-end artifacts in one GPU call (stops at the first failure): the whole -m gpu suite and smoke();
# PMC traffic / issue passes -> profiles/$ROUND/traffic.json, the rocprofv3 kernel-trace stats of the
# default bench and the default bench itself (scripts/round_artifacts.sh); every BASELINE config and the
# large values (scripts/gpu_configs.sh).
#   ROUND=r06 TAG=r6final bash scripts/gpu_final.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r06}
TAG=${TAG:-final}
TAG=$TAG/suite bash scripts/gpu_suite.sh || exit $?
ROUND=$ROUND TAG=$TAG/art bash scripts/round_artifacts.sh || exit $?
TAG=$TAG/configs bash scripts/gpu_configs.sh || exit $?
