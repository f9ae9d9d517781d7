set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python -u tools/fc_ablate.py 0,16 > gpurun_out/fc_ablate.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_wal.json 2> gpurun_out/bench_wal.err
timeout -k 10 300 python -u bench.py --workload shards --no-cpu-baseline > gpurun_out/bench_shards.json 2> gpurun_out/bench_shards.err
