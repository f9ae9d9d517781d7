# Round-2 final measurement, part 2: bench + rocprof stats for snap / commit / msg / snapstream / restart
set -e
mkdir -p gpurun_out
bash tools/bench_all.sh snap commit msg snapstream restart > gpurun_out/final_bench_b.log 2>&1
