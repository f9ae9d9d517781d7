#!/bin/bash
# Round-5 session 10: A/B of the half-line k_stream loads (one permlane32
# stage) and the frame pass's prefix ablations (timing only: EW_FR_ABL 1 no
# Horner over v, 2 no prefix tail, 4 no S_dlen -- verdicts wrong by design).
set -eo pipefail
out=${1:-gpurun_out/s10}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_new.so ablibs/libewal_half.so > "$out/ab_half_wal.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py shards 2 ablibs/libewal_new.so ablibs/libewal_half.so > "$out/ab_half_shards.txt" 2>&1
AB_NOCHECK=1 timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_new.so ablibs/libewal_abl1.so \
  ablibs/libewal_abl2.so ablibs/libewal_abl4.so > "$out/ab_fr_abl_c1.txt" 2>&1
AB_NOCHECK=1 timeout -k 10 600 python3 tools/ab_run.py wal 2 ablibs/libewal_new.so ablibs/libewal_abl1.so \
  ablibs/libewal_abl2.so ablibs/libewal_abl4.so > "$out/ab_fr_abl_wal.txt" 2>&1
echo done
