#!/bin/bash
# Round-5 session 19: v[] / hmask stored nontemporally by the stream pass (the
# 11-12 us between k_stream's end and k_frames' start in the kernel trace).
set -eo pipefail
out=${1:-gpurun_out/s19}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_base.so ablibs/libewal_vnt.so > "$out/ab_vnt_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_base.so ablibs/libewal_vnt.so > "$out/ab_vnt_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_base.so ablibs/libewal_vnt.so ablibs/libewal_segcall.so \
  > "$out/ab_vnt_shards.txt" 2>&1
echo done
