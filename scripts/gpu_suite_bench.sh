cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/g1/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/g1/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err; rc=$?
cat gpurun_out/g1/bench.json; exit $rc
