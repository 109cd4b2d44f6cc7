#!/bin/bash
# Every BASELINE size plus the large values (30 KB, 64 KiB, 1 MiB) on the current kernels, with the
# reference digest match of each leg (fullsize_parity).  Stops at the first failure.
#   TAG=r6cfg bash scripts/gpu_configs.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-cfg}
mkdir -p gpurun_out/$T
run() { # name, args...
  local name=$1; shift
  timeout -k 10 ${TLIM:-300} python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/$name.json 2> gpurun_out/$T/$name.err || return $?
  python3 scripts/bench_line.py gpurun_out/$T/$name.json $name
}
run b256 --vlen 256 &&
run b4k --n 1000000 --vlen 4096 &&
run alnum --n 1000000 --kind 1 &&
timeout -k 10 300 python bench.py --mix > gpurun_out/$T/mix.json 2> gpurun_out/$T/mix.err && cat gpurun_out/$T/mix.json &&
run h2h --h2h &&
python3 -c "import json;d=json.load(open('gpurun_out/$T/h2h.json'))['host_to_host'];print('h2h',d['pipelined'])" &&
run b30k --n 100000 --vlen 30000 --steps 2 &&
run b64k --n 40000 --vlen 65536 --steps 2 &&
TLIM=400 run b1m --n 1000 --vlen 1048576 --steps 1
