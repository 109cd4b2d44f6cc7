#!/bin/bash
# iteration run: parity tests, per-phase instruction counts, stamps, bench (stops on first failure)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-iter}
timeout -k 10 900 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
TAG=${TAG}_phase bash scripts/phase_cost.sh > gpurun_out/${TAG}_phase.log 2>&1
rc=$?; echo "phase rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
exit $rc
