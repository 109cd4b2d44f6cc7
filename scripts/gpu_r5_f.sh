#!/bin/bash
# Round 5: inflate_rec phase times on the byte-list kernel (stop build), then the 30 KB routing A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5f}
O=gpurun_out/$T
mkdir -p $O
for st in 31 32 -1; do
  PMC_LIB=libpmc_codec_stop.so PMC_STOP_AFTER=$st timeout -k 10 200 python scripts/rec_phase_time.py 4000000 1024 >> $O/rec_phase.jsonl 2> $O/rec_phase.err || exit $?
done
python3 -c "
import json
for l in open('$O/rec_phase.jsonl'): d=json.loads(l); print(d['stop_after'], round(d['ms_per_launch']['inflate_rec'],2))"
TAG=r5big bash scripts/gpu_r5_big.sh
