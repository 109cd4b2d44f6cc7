cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ft
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/ft/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/ft/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ft/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/ft/smoke.log
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ft/server bash scripts/server_bench.sh > gpurun_out/ft/server.txt 2>&1; rc=$?
echo "server rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/latency_dropin.py > gpurun_out/ft/latency.json 2> gpurun_out/ft/latency.err; echo "latency rc=$?"
