#!/bin/bash
# iteration run: parity tests, stamps, bench (stops on the first failure/fault)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-iter}
timeout -k 10 900 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
PMC_LIB=libpmc_codec_stamps.so timeout -k 10 300 python scripts/stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/${TAG}_stamps.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
exit $rc
