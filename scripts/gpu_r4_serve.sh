#!/bin/bash
# Round 4 server-shaped batches: kernel trace of bench.py --batches (where a small batch's time goes),
# the batch leg itself, and the reference server + hook at 1 KiB with the SET batch asynchronous
# (default) and synchronous (PMC_HOOK_SYNC=1), recording a server that ends under load.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4serve}
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv \
    -- python3 bench.py --batches > gpurun_out/$T/batches_traced.json 2> gpurun_out/$T/batches_traced.err || exit $?
timeout -k 10 300 python bench.py --batches > gpurun_out/$T/batches.json 2> gpurun_out/$T/batches.err || exit $?
cat gpurun_out/$T/batches.json
for mode in async sync; do
  if [ $mode = sync ]; then export PMC_HOOK_SYNC=1; fi
  OUT=gpurun_out/$T/refsrv_$mode SHAPES="1024 16 8192 40000
4096 16 8192 40000" SERVERS="ref_batch" timeout -k 10 400 bash scripts/ref_server_bench.sh > gpurun_out/$T/refsrv_$mode.log 2>&1
  echo "$mode rc=$?"; tail -4 gpurun_out/$T/refsrv_$mode.log | cut -c1-300
  grep -h "exited with status" gpurun_out/$T/refsrv_$mode/server_*.log
done
exit 0
