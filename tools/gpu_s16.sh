#!/bin/bash
# Round-5 session 16: the unit lins from the stream pass (EW_ULIN: the frame
# pass's phase A loads one dword per unit instead of a Horner over 16 v[]):
# the GPU suite, then A/B against the same build without them.
set -eo pipefail
out=${1:-gpurun_out/s16}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_noulin.so ablibs/libewal_ulin.so > "$out/ab_ulin_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_noulin.so ablibs/libewal_ulin.so > "$out/ab_ulin_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_noulin.so ablibs/libewal_ulin.so > "$out/ab_ulin_shards.txt" 2>&1
echo done
