#!/bin/bash
# Round 5: device-resident batches of <= 1,024 small values on the one-kernel paths -- the whole -m gpu
# suite, then the batch table.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5small}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
PMC_HOST_TRACE=1 timeout -k 10 300 python bench.py --batches > $O/batches.json 2> $O/batches.err || exit $?
python3 - $O/batches.json <<'PY'
import json, sys
for b in json.load(open(sys.argv[1]))["batches"]:
    print(b["values"], {k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in b.items() if k.endswith("_ms")}, b["mismatches"])
PY
