#!/bin/bash
# Round-5 session 6: the GPU suite, then the default bench line and the
# restart E2E line (each its own process).  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s6}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
timeout -k 10 300 python3 bench.py --workload restart --steps 3 --warmup 1 > "$out/restart.json" 2> "$out/restart.err"
echo done
