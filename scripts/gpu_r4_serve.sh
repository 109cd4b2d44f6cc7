#!/bin/bash
# Round 4 server-shaped batches: kernel trace of bench.py --batches (where a small batch's time goes),
# the batch leg itself, and the reference server + hook at 1 and 4 KiB with the SET batch
# synchronous (default) and asynchronous (PMC_HOOK_ASYNC=1), recording a server that ends under load.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4serve}
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv \
    -- python3 bench.py --batches > gpurun_out/$T/batches_traced.json 2> gpurun_out/$T/batches_traced.err || exit $?
timeout -k 10 300 python bench.py --batches > gpurun_out/$T/batches.json 2> gpurun_out/$T/batches.err || exit $?
timeout -k 10 300 python bench.py --batches --batch-vlen 1024 > gpurun_out/$T/batches_1k.json 2> gpurun_out/$T/batches_1k.err || exit $?
PMC_DEFLATE_MONO=1 timeout -k 10 300 python bench.py --batches --batch-vlen 1024 > gpurun_out/$T/batches_1k_mono.json 2> gpurun_out/$T/batches_1k_mono.err || exit $?
PMC_INFLATE_WAVE=1 timeout -k 10 300 python bench.py --batches --batch-vlen 1024 > gpurun_out/$T/batches_1k_wave.json 2> gpurun_out/$T/batches_1k_wave.err || exit $?
python3 - gpurun_out/$T <<'PY'
import json, sys
for f in ("batches", "batches_1k", "batches_1k_mono", "batches_1k_wave"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    for b in d["batches"]:
        print(f, b["values"], b["value_bytes"], {k: round(v, 3) for k, v in b["device_ms"].items()},
              {k: round(v, 3) for k, v in b["host_ms"].items()}, b["mismatches"])
PY
for mode in sync async; do
  if [ $mode = async ]; then export PMC_HOOK_ASYNC=1; fi
  OUT=gpurun_out/$T/refsrv_$mode SHAPES="1024 16 8192 40000
4096 16 8192 40000" SERVERS="ref_batch" timeout -k 10 400 bash scripts/ref_server_bench.sh > gpurun_out/$T/refsrv_$mode.log 2>&1
  echo "$mode rc=$?"; tail -4 gpurun_out/$T/refsrv_$mode.log | cut -c1-300
  grep -h "exited with status" gpurun_out/$T/refsrv_$mode/server_*.log
done
exit 0
