#!/bin/bash
# Round 4: the large-value path -- its parity tests, the guard tests, the codec suite's large cases,
# then 40K x 64 KiB and 1000 x 1 MiB JSON-slice benches (compress + decompress, every value verified).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r4large}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_large.txt 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_large.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_guard.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_guard.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -v -k "golden or ragged or multi_megabyte" --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_codec.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_codec.txt; [ $rc -eq 0 ] || exit $rc
for cfg in "40000 65536" "1000 1048576" "100000 30000"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --n $1 --vlen $2 --steps 2 > gpurun_out/$T/b_$2.json 2> gpurun_out/$T/b_$2.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/$T/b_$2.json'));print('$2',d['value'],d['compress_gib_s'],d['decompress_gib_s'],d['mismatches'],d['roofline']['kernel_ms_per_step'])"
done
# server-shaped batches: the default routing, then the wave-per-member inflate for comparison
timeout -k 10 300 python bench.py --batches > gpurun_out/$T/batches.json 2> gpurun_out/$T/batches.err || exit $?
PMC_INFLATE_WAVE=1 timeout -k 10 300 python bench.py --batches > gpurun_out/$T/batches_wave.json 2> gpurun_out/$T/batches_wave.err || exit $?
PMC_DEFLATE_MONO=1 timeout -k 10 300 python bench.py --batches > gpurun_out/$T/batches_mono.json 2> gpurun_out/$T/batches_mono.err || exit $?
cat gpurun_out/$T/batches.err gpurun_out/$T/batches_wave.err gpurun_out/$T/batches_mono.err
OUT=gpurun_out/$T/refsrv timeout -k 10 600 bash scripts/ref_server_bench.sh > gpurun_out/$T/refsrv.log 2>&1; rc=$?
tail -12 gpurun_out/$T/refsrv.log; exit $rc
