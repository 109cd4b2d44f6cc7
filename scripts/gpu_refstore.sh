#!/bin/bash
# Round-6 f2 inside the reference's own kvs: the reference-server GPU tests (dropin, batch, store), then the
# hook with and without the device store beside pmc_server under the same load.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_refstore.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6store
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_ref_server.py > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
OUT=$OUT/bench SERVERS="ref_batch ref_store pmc_batch" SHAPES="4096 64 65536 100000
1024 16 8192 40000" timeout -k 10 400 bash scripts/ref_server_bench.sh
