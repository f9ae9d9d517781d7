set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_wal.py tests/test_gpu_shim.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --workload restart --steps 3 > gpurun_out/bench_restart.json 2> gpurun_out/bench_restart.err
timeout -k 10 400 python -u tools/fc_ablate.py > gpurun_out/fc_ablate.log 2>&1
