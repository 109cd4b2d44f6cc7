#!/bin/bash
# A/B iteration run: GPU parity tests, then the default bench with and without an env toggle.
#   TAG=x AB_ENV="PMC_DEFLATE_MONO=1" bash scripts/gpu_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_a.json 2> gpurun_out/${TAG}_bench_a.err
rc=$?; echo "bench A rc=$rc"; cat gpurun_out/${TAG}_bench_a.json
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_b.json 2> gpurun_out/${TAG}_bench_b.err
  rc=$?; echo "bench B ($AB_ENV) rc=$rc"; cat gpurun_out/${TAG}_bench_b.json
fi
exit $rc
