set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tools/bench_all.sh wal c1 shards snap commit msg restart snapstream > gpurun_out/bench_all.log 2>&1
