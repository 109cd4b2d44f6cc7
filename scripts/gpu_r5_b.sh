#!/bin/bash
# Round 5: inflate_rec phase times (stop build) and the host-batch legs after the copy-thread change.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5b}
O=gpurun_out/$T
mkdir -p $O
for st in 31 32 -1; do
  PMC_LIB=libpmc_codec_stop.so PMC_STOP_AFTER=$st timeout -k 10 200 python scripts/rec_phase_time.py 4000000 1024 >> $O/rec_phase.jsonl 2> $O/rec_phase.err || exit $?
done
cat $O/rec_phase.jsonl
PMC_HOST_TRACE=1 timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
grep -v pmc_host_trace $O/batches.err | cut -c1-400
