#!/bin/bash
# Parity + same-box A/B of the working tree's build (B) against HEAD (A); TAG names the output.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s8_ab}
mkdir -p gpurun_out/$T
TAG=$T/ab bash scripts/ab_check.sh
