#!/bin/bash
# Round-5 session 13: the host side of one ReadAll call -- blocking wait vs a
# spin on the stream (EWAL_SPIN), with and without the markers between the
# kernels (EWAL_NO_MID_EVENTS) -- hooks build, one box.
set -eo pipefail
out=${1:-gpurun_out/s13}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/host_gap.py c1 3 ablibs/libewal_hooks2.so X=0 EWAL_SPIN=1 EWAL_NO_MID_EVENTS=1 \
  EWAL_SPIN=1+EWAL_NO_MID_EVENTS=1 > "$out/host_gap_c1.txt" 2>&1
timeout -k 10 600 python3 tools/host_gap.py wal 2 ablibs/libewal_hooks2.so X=0 EWAL_SPIN=1 EWAL_NO_MID_EVENTS=1 \
  EWAL_SPIN=1+EWAL_NO_MID_EVENTS=1 > "$out/host_gap_wal.txt" 2>&1
echo done
