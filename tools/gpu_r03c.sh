#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 100 python -u tools/dbg_batch.py > $OUT/dbg_N.txt 2>&1; echo "dbg N rc=$?"
EWAL_LIB_PATH=ablibs/libewal_A.so timeout -k 10 100 python -u tools/dbg_batch.py > $OUT/dbg_A.txt 2>&1; echo "dbg A rc=$?"
EWAL_FUSED=0 timeout -k 10 100 python -u tools/dbg_batch.py > $OUT/dbg_nofused.txt 2>&1; echo "dbg nofused rc=$?"
AB_NOCHECK=1 timeout -k 10 400 python -u tools/ab_run.py shards 2 ablibs/libewal_N.so ablibs/libewal_X2.so ablibs/libewal_X4.so ablibs/libewal_X6.so > $OUT/ab_shards.txt 2>&1; echo "ab shards rc=$?"
AB_NOCHECK=1 timeout -k 10 300 python -u tools/ab_run.py wal 2 ablibs/libewal_A.so ablibs/libewal_N.so ablibs/libewal_X2.so ablibs/libewal_X4.so > $OUT/ab_wal.txt 2>&1; echo "ab wal rc=$?"
