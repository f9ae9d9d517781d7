set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dir.py tests/test_gpu_shim.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --workload restart --steps 3 > gpurun_out/bench_restart.json 2> gpurun_out/bench_restart.err
