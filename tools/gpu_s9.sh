#!/bin/bash
# Round-5 session 9: the GPU suite on the k_stream instruction cuts (one-step
# super-piece lins, 32-bit borrow tests, the pair loop without bounds tests)
# and the seam's wave-level fold, then A/B against the previous build and the
# seam / fr_result step timing.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s9}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_base.so ablibs/libewal_new.so ablibs/libewal_notree.so \
  > "$out/ab_wal.txt" 2>&1
timeout -k 10 300 python3 tools/ab_run.py c1 3 ablibs/libewal_base.so ablibs/libewal_new.so > "$out/ab_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_base.so ablibs/libewal_new.so > "$out/ab_shards.txt" 2>&1
EWAL_LIB_PATH=ablibs/libewal_tm.so timeout -k 10 300 python3 tools/fr_timing.py > "$out/fr_timing.txt" 2>&1
echo done
