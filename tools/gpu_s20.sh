#!/bin/bash
# Round-5 session 20: A/B: v[] / hmask stored nontemporally, and the batch kernel with the
# stream-end prefix call (fewer spills in k_frames<true, ...>).
set -eo pipefail
out=${1:-gpurun_out/s20}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_base.so ablibs/libewal_vnt.so ablibs/libewal_segcall.so \
  > "$out/ab_shards.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_base.so ablibs/libewal_vnt.so > "$out/ab_vnt_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_base.so ablibs/libewal_vnt.so > "$out/ab_vnt_c1.txt" 2>&1
echo done
