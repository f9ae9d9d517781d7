#!/bin/bash
# r03 GPU call b: debug + batch/parity tests + A/B timing (near prefix, candidate ablations)
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 100 python -u tools/dbg_batch.py > $OUT/dbg.txt 2>&1; echo "dbg rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_framing.py -q --timeout 120 --timeout-method thread > $OUT/pytest_part.txt 2>&1; echo "pytest rc=$?"
tail -5 $OUT/pytest_part.txt
AB_NOCHECK=1 timeout -k 10 300 python -u tools/ab_run.py shards 2 ablibs/libewal_A.so ablibs/libewal_N.so ablibs/libewal_X2.so > $OUT/ab_shards.txt 2>&1; echo "ab shards rc=$?"
tail -3 $OUT/ab_shards.txt
AB_NOCHECK=1 timeout -k 10 300 python -u tools/ab_run.py wal 2 ablibs/libewal_A.so ablibs/libewal_N.so > $OUT/ab_wal.txt 2>&1; echo "ab wal rc=$?"
tail -2 $OUT/ab_wal.txt
