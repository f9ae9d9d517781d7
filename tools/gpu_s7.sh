#!/bin/bash
# Round-5 session 7: the GPU suite, the default bench line and the restart E2E
# line (each its own process), then k_frames wave end times and a frame-grid
# sweep.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s7}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
timeout -k 10 300 python3 bench.py --workload restart --steps 3 --warmup 1 > "$out/restart.json" 2> "$out/restart.err"
EWAL_LIB_PATH=ablibs/libewal_tm.so timeout -k 10 300 python3 tools/fr_timing.py > "$out/fr_timing.txt" 2>&1
timeout -k 10 600 python3 tools/env_sweep.py wal 2 ablibs/libewal_hooks.so X=0 EWAL_FRAME_CUS=228 \
  EWAL_FRAME_CUS=205 EWAL_FRAME_CUS=256 > "$out/sweep_frame_grid.txt" 2>&1
echo done
