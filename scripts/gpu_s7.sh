#!/bin/bash
# Wide lane-inflate pass: probe + parity + A/B (default and 100K x 30 KB), then the reference server bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-s7}
mkdir -p gpurun_out/$T
PMC_LIB=libpmc_codec_alt.so timeout -k 10 300 python3 scripts/inflate_probe.py 30000 16000 8192 > gpurun_out/$T/probe.txt 2>&1; rc=$?
cat gpurun_out/$T/probe.txt
[ $rc -eq 0 ] || exit $rc
TAG=$T/ab bash scripts/ab_check.sh || exit $?
TAG=$T/ab30k BENCH_ARGS="--n 100000 --vlen 30000" bash scripts/gpu_abab.sh || exit $?
OUT=gpurun_out/$T/refsrv timeout -k 10 900 bash scripts/ref_server_bench.sh > gpurun_out/$T/refsrv.log 2>&1; rc=$?
tail -8 gpurun_out/$T/refsrv.log
exit $rc
