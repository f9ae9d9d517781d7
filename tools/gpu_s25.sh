#!/bin/bash
# Round-5 session 25: 8-unit (32 KiB) tiles for the smallest streams:
# the GPU suite (small WALs now take the 8-unit tiles), the empty-tile
# regression on the 16-unit build, then A/B on configs[0].
set -eo pipefail
out=${1:-gpurun_out/s25}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
EWAL_LIB_PATH=$PWD/ablibs/libewal_notsh3.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_configs.py -m gpu -k "tiles_without or leader_changes" > "$out/pytest_notsh3.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 5 ablibs/libewal_notsh3.so ablibs/libewal_tsh3.so > "$out/ab_tsh3_c1.txt" 2>&1
echo done
