#!/bin/bash
# Round 4: where the large-value compressor's time goes (kernel trace of 40K x 64 KiB and 1000 x 1 MiB).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4lvprof}
mkdir -p gpurun_out/$T
for cfg in "40000 65536" "1000 1048576"; do
  set -- $cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/p$2 -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --n $1 --vlen $2 --steps 1 --warmup 1 > gpurun_out/$T/b_$2.json 2> gpurun_out/$T/b_$2.err || exit $?
  python3 - gpurun_out/$T/p$2/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(r["Name"][:50].ljust(50), r["Calls"].rjust(5), "%10.2f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
done
