#!/bin/bash
# sizing run, full default bench, then a rocprofv3 kernel-trace of a reduced run
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python bench.py --n 1000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.err
rc=$?; echo "bench_1m rc=$rc"; cat gpurun_out/bench_1m.json; tail -3 gpurun_out/bench_1m.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench_full rc=$rc"; cat gpurun_out/bench_full.json; tail -3 gpurun_out/bench_full.err
if fatal $rc; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run -f csv -- python3 bench.py --n 2000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_r1.log
find gpurun_out/prof_r1 -name "*stats*" | head
exit $rc
