#!/bin/bash
# Round-5 session 23: the seam pass with two threads per tile -- the GPU suite,
# then A/B against one thread per tile.
set -eo pipefail
out=${1:-gpurun_out/s23}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_nosplit.so ablibs/libewal_split.so > "$out/ab_split_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_nosplit.so ablibs/libewal_split.so > "$out/ab_split_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_nosplit.so ablibs/libewal_split.so > "$out/ab_split_shards.txt" 2>&1
echo done
