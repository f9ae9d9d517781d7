set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-seconds 4 > gpurun_out/bench_wal.json 2> gpurun_out/bench_wal.err
timeout -k 10 300 python -u bench.py --workload restart --steps 3 > gpurun_out/bench_restart.json 2> gpurun_out/bench_restart.err
timeout -k 10 400 python -u bench.py --workload snapstream > gpurun_out/bench_snapstream.json 2> gpurun_out/bench_snapstream.err
