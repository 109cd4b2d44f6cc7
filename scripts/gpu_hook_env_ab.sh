#!/bin/bash
# A B A B of the f1 hook (ref_server_batch, 4 KiB / 64 connections) with the latency path on (default) and off
# (PMC_LATENCY_BATCH=0: every batch through the throughput pipeline).
cd "$GRAFT_REPO_ROOT" || exit 1
for k in 1 2; do
  for v in default 0; do
    if [ $v = default ]; then unset PMC_LATENCY_BATCH; else export PMC_LATENCY_BATCH=$v; fi
    OUT=gpurun_out/r6hookab/lat_${v}_$k SERVERS="ref_batch" SHAPES="4096 64 65536 100000" \
        timeout -k 10 200 bash scripts/ref_server_bench.sh > /dev/null 2>&1
    echo "lat=$v run=$k $(tail -1 gpurun_out/r6hookab/lat_${v}_$k/ref_server_bench.jsonl)"
  done
done
