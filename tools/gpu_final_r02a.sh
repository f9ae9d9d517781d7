# Round-2 final measurement, part 1: GPU suite, smoke, k_stream traffic PMC, bench + rocprof stats for wal / c1 / shards
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final_pytest_gpu.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1
bash tools/traffic.sh gpurun_out/traffic
bash tools/bench_all.sh wal c1 shards > gpurun_out/final_bench_a.log 2>&1
