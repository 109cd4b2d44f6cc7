#!/bin/bash
# Loopback ops/s of the reference's OWN CacheServer (oracle/_ref/ref_server_*: src/server + kvs
# compiled unmodified) under pmc_loadgen (BASELINE configs[4] shape: pipelined batches of 100 commands
# per connection, 4 KiB JSON-slice values, 50 % SET, every GET checked), beside pmc_server:
#   zlib    the reference as deployed: its gzip_compressor.cpp + zlib on the single request thread
#           (server.cpp:631-643) -- the CPU baseline of this config, timed on this host
#   dropin  the drop-in GzipCompressor, one GPU call per value
#   batch   the drop-in + the f1 batch hook (one device batch per direction per epoll iteration)
#   store   the batch build with kvs holding compressed values in HBM (f2, ref_store_hook.cpp)
#   nocodec the same server with ENABLE_COMPRESSION=false: its request path alone
# No connection before a server prints its ready line; pmc_loadgen then waits (10 s) until it answers
# and writes 20 ms after connecting, which keeps clear of the reference's connect race (INTEGRATION.md
# 3.2.1: conn_manager.hpp:83-93, server.cpp:373,409).  A reference server that never answers has
# self-deadlocked (validateConnections -> closeConnection relocks conn_mutex, conn_manager.hpp:117, :142;
# about half of all starts on a long-running host): it is killed and started again, at most five times.
# PROTO=resp sends every command as a RESP array (both servers speak it; server.cpp:147-280).
#   OUT=gpurun_out/x bash scripts/ref_server_bench.sh
cd "$GRAFT_REPO_ROOT" || cd "$(dirname "$0")/.." || exit 1
OUT=${OUT:-gpurun_out/refsrv}
mkdir -p "$OUT"
B=poor-man-s-cache_amd/pmc_codec
once() {  # tag cmd... : start a server (cmd), run the load, stop it
    local tag=$1; shift
    local port=$((20000 + RANDOM % 20000))
    "$@" $port > "$OUT/server_$tag.log" 2>&1 &
    local pid=$!
    # no connection before the server's Start() prints its ready line (connections queued in the backlog
    # meanwhile are accepted together, inside the reference's connect race)
    for k in $(seq 1 600); do grep -q "ready to accept\|READY" "$OUT/server_$tag.log" 2>/dev/null && break; sleep 0.1; done
    timeout -k 5 240 $B/pmc_loadgen --port $port --data tests/golden/data --vlen $VLEN --ops $OPS --conns $CONNS \
        --keys $KEYS --batch 100 --mix 50 --warmup-sec 10 --proto ${PROTO:-custom} > "$OUT/load_$tag.json" 2> "$OUT/load_$tag.err"
    local rc=$?
    # (the no-codec leg: GET answers a pointer into the store, kvs.cpp:224, which a later SET of the same
    # key in the same epoll iteration frees before the responses go out -- a reference defect the codec
    # hides by answering a fresh copy; its mismatches are recorded, not failed)
    if [ $rc -eq 1 ] && [ -n "$ALLOW_MISMATCH" ] && grep -q '"failed_conns": 0' "$OUT/load_$tag.json" 2>/dev/null; then rc=0; fi
    if ! kill -0 $pid 2>/dev/null; then  # the server ended under the load: record how
        wait $pid; echo "server $tag exited with status $? during the load" | tee -a "$OUT/server_$tag.log"
        return $rc
    fi
    kill $pid; sleep 2; kill -9 $pid 2>/dev/null; wait $pid 2>/dev/null
    return $rc
}
ref_server() { SERVER_PORT=$2 NUM_SHARDS=128 PMC_PRIME_STATS="$OUT/prime_$1_${VLEN}_${CONNS}.json" oracle/_ref/ref_server_$1; }
# the reference's request path with no codec at all (ENABLE_COMPRESSION=false, main.cpp:22): the ceiling
# of any codec under it, the hook included
ref_nocodec() { SERVER_PORT=$2 NUM_SHARDS=128 ENABLE_COMPRESSION=false oracle/_ref/ref_server_zlib; }
pmc_srv() { $B/pmc_server --port $2 --codec $1 --heap-mb 8192; }
case_() {  # label server-fn kind
    local tag="$1_${VLEN}_${CONNS}_${KEYS}_${PROTO:-custom}"
    for attempt in 1 2 3 4 5; do
        if once "$tag" $2 $3; then
            sed "s/^{/{\"server\": \"$1\", \"attempt\": $attempt, /" "$OUT/load_$tag.json" | tee -a "$OUT/ref_server_bench.jsonl"
            return 0
        fi
        grep -q "did not answer" "$OUT/load_$tag.err" || { cat "$OUT/load_$tag.err"; return 1; }
    done
    echo "{\"server\": \"$1\", \"failed\": \"no answer after 5 starts\", \"vlen\": $VLEN, \"conns\": $CONNS}" | tee -a "$OUT/ref_server_bench.jsonl"
}
# (SHAPES / SERVERS narrow the run, e.g. SHAPES="1024 16 8192 40000" SERVERS="ref_batch")
SERVERS=${SERVERS:-ref_zlib ref_nocodec ref_batch pmc_batch pmc_off ref_dropin}
want() { case " $SERVERS " in *" $1 "*) return 0 ;; esac; return 1; }
while read -r shape; do
    [ -n "$shape" ] || continue
    set -- $shape
    VLEN=$1 CONNS=$2 KEYS=$3 OPS=$4
    if want ref_zlib; then case_ ref_zlib ref_server zlib || exit 1; fi
    if want ref_nocodec; then ALLOW_MISMATCH=1 case_ ref_nocodec ref_nocodec none || exit 1; fi
    if want ref_batch; then case_ ref_batch ref_server batch || exit 1; fi
    if want ref_store; then case_ ref_store ref_server store || exit 1; fi
    if want pmc_batch; then case_ pmc_batch pmc_srv batch || exit 1; fi
    if want pmc_off; then case_ pmc_off pmc_srv off || exit 1; fi
done <<< "${SHAPES:-4096 16 8192 40000
4096 64 65536 100000
1024 16 8192 40000}"
if want ref_dropin; then VLEN=4096 CONNS=16 KEYS=1024 OPS=4000 case_ ref_dropin ref_server dropin; fi
exit 0
