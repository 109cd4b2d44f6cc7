#!/bin/bash
# Round 5: per-kernel times of the large-value legs (kernel trace only).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5lvt}
O=gpurun_out/$T
mkdir -p $O
for cfg in "100000 30000" "40000 65536"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$2 -o run -f csv -- python3 bench.py --no-cpu-baseline \
      --n $1 --vlen $2 --steps 1 --warmup 1 > $O/b_$2.json 2> $O/b_$2.err || exit $?
  python3 - $O/t_$2/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"].split("(")[0][:40]:40s} calls {r["Calls"]:>4s} total {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
done
