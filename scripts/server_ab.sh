#!/bin/bash
# Loopback server runs under two environments (A, then B="$ENV_B"), twice each: what a codec policy
# switch does to small server batches.   ENV_B="PMC_REC_MIN_N=100000" bash scripts/server_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-sab}
mkdir -p "$OUT"
B=poor-man-s-cache_amd/pmc_codec
run() {  # label vlen conns mix
    local port=$((20000 + RANDOM % 20000))
    env ${5:-} $B/pmc_server --port $port --codec batch --heap-mb 8192 > "$OUT/server_$1.log" 2>&1 &
    local pid=$!
    sleep 1
    timeout -k 5 200 $B/pmc_loadgen --port $port --data tests/golden/data --vlen $2 --ops 400000 --conns $3 \
        --keys 65536 --batch 100 --mix $4 | sed "s/^{/{\"label\": \"$1\", /" | tee -a "$OUT/runs.jsonl"
    local rc=${PIPESTATUS[0]}
    kill $pid; wait $pid
    return $rc
}
for r in 1 2; do
  run A1k 1024 64 50 && run B1k 1024 64 50 "$ENV_B" && run A4kget 4096 64 0 && run B4kget 4096 64 0 "$ENV_B" &&
  run A4k 4096 64 50 && run B4k 4096 64 50 "$ENV_B" || exit 1
done
