#!/bin/bash
# Loopback ops/s of the reference's OWN CacheServer (oracle/_ref/ref_server_*: src/server + kvs
# compiled unmodified) under pmc_loadgen (BASELINE configs[4] shape: pipelined batches of 100 commands
# per connection, 4 KiB JSON-slice values, 50 % SET), beside pmc_server:
#   (the reference server itself stops answering under some of these loads -- its zlib build at 16
#   connections in the build container, its batch build at 65,536 keys on the GPU box: no answer within
#   60 s -- so the runs use the shape the GPU tests pass with: 16 connections, 8,192 keys)
#   dropin  the drop-in GzipCompressor, one GPU call per value
#   batch   the drop-in + the f1 batch hook (one device batch per direction per epoll iteration)
#   OUT=gpurun_out/x bash scripts/ref_server_bench.sh
cd "$GRAFT_REPO_ROOT" || cd "$(dirname "$0")/.." || exit 1
OUT=${OUT:-gpurun_out/refsrv}
mkdir -p "$OUT"
B=poor-man-s-cache_amd/pmc_codec
run() {  # kind vlen ops conns mix keys
    local port=$((20000 + RANDOM % 20000))
    SERVER_PORT=$port NUM_SHARDS=128 PMC_PRIME_STATS="$OUT/prime_$1_$2_$4_$5.json" \
        oracle/_ref/ref_server_$1 > "$OUT/server_$1_$2_$4_$5.log" 2>&1 &
    local pid=$!
    sleep 1
    timeout -k 5 240 $B/pmc_loadgen --port $port --data tests/golden/data --vlen $2 --ops $3 --conns $4 \
        --keys $6 --batch 100 --mix $5 | sed "s/^{/{\"server\": \"ref_$1\", /" | tee -a "$OUT/ref_server_bench.jsonl"
    local rc=${PIPESTATUS[0]}
    kill $pid; sleep 2; kill -9 $pid 2>/dev/null; wait $pid
    return $rc
}
pmc() {  # codec vlen ops conns mix keys
    local port=$((20000 + RANDOM % 20000))
    $B/pmc_server --port $port --codec $1 --heap-mb 8192 > "$OUT/pmc_$1_$2_$4_$5.log" 2>&1 &
    local pid=$!
    sleep 1
    timeout -k 5 240 $B/pmc_loadgen --port $port --data tests/golden/data --vlen $2 --ops $3 --conns $4 \
        --keys $6 --batch 100 --mix $5 | sed "s/^{/{\"server\": \"pmc_$1\", /" | tee -a "$OUT/ref_server_bench.jsonl"
    local rc=${PIPESTATUS[0]}
    kill $pid; sleep 2; kill -9 $pid 2>/dev/null; wait $pid
    return $rc
}
run batch 4096 40000 16 50 8192 &&
pmc batch 4096 40000 16 50 8192 &&
run dropin 4096 4000 16 50 1024 &&
run batch 1024 40000 16 50 8192 &&
pmc batch 1024 40000 16 50 8192
