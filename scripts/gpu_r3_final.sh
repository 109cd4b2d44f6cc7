#!/bin/bash
# Round-3 final: PMC traffic/issue + traced bench + default bench on the final sources, the GPU suite, smoke,
# then the BASELINE configs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROUND=r03 TAG=r3final3 bash scripts/round_artifacts.sh || exit $?
T=r3final3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.txt 2>&1; rc=$?
tail -2 gpurun_out/$T/smoke.txt; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/$name.json 2> gpurun_out/$T/$name.err || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value'],3),round(d['compress_gib_s'],3),round(d['decompress_gib_s'],3),d['mismatches'])" gpurun_out/$T/$name.json $name
}
run b256 --vlen 256 && run b4k --n 1000000 --vlen 4096 && run alnum --n 1000000 --kind 1 &&
timeout -k 10 300 python bench.py --mix > gpurun_out/$T/mix.json 2> gpurun_out/$T/mix.err && tail -c 400 gpurun_out/$T/mix.json &&
run h2h --h2h && python3 -c "import json;print(json.load(open('gpurun_out/$T/h2h.json'))['host_to_host']['pipelined'])"
