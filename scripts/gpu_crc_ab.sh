cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "crc32 or decompress or ragged or roundtrip or digest" > gpurun_out/crc_pytest.log 2>&1 && \
TAG=crc bash scripts/gpu_abab.sh
