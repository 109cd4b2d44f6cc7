#!/bin/bash
# Round-6 RESP leg of f1/f3 on the GPU box: the store's per-extent frames and both pmc_server codecs in RESP
# (tests), then pmc_server and the reference over zlib under the same load in custom and RESP framing.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_resp.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6resp
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_store.py tests/test_server.py > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
for proto in custom resp; do
    OUT=$OUT/bench PROTO=$proto SERVERS="pmc_batch ref_zlib" SHAPES="4096 64 65536 100000" \
        timeout -k 10 300 bash scripts/ref_server_bench.sh || exit 1
done
