set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python -u tools/first_call.py > gpurun_out/first_call.log 2>&1
timeout -k 10 200 python -u bench.py --cpu-seconds 2 > gpurun_out/bench.log 2>&1
BENCH_ARGS="--workload shards --shards-per-gpu 128" 
tools/pmc_stream.sh gpurun_out/pmc_shards --workload shards --shards-per-gpu 128 > gpurun_out/pmc.log 2>&1
