#!/bin/bash
# Round-5 session 15: the stream-end prefix from the frame pass (the seam's
# slowest thread stepped up to 255 bytes through global tables): the GPU suite,
# A/B against the previous build, the seam step timing.
set -eo pipefail
out=${1:-gpurun_out/s15}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_prev.so ablibs/libewal_peb.so > "$out/ab_peb_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_prev.so ablibs/libewal_peb.so > "$out/ab_peb_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_prev.so ablibs/libewal_peb.so > "$out/ab_peb_shards.txt" 2>&1
EWAL_LIB_PATH=ablibs/libewal_tm.so timeout -k 10 300 python3 tools/fr_timing.py > "$out/fr_timing.txt" 2>&1
echo done
