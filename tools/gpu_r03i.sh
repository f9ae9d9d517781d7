#!/bin/bash
# r03 call i: GPU suite on the hybrid candidate tests (k_stream inline for sparse units, k_cand for the rest), A/B vs HEAD
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -3 $OUT/pytest.txt
grep -q passed $OUT/pytest.txt && ! grep -q failed $OUT/pytest.txt || exit 1
step timeout -k 10 300 python -u tools/ab_run.py wal 3 ablibs/libewal_N.so ablibs/libewal_I0.so ablibs/libewal_I2.so ablibs/libewal_I4.so > $OUT/ab_wal.txt 2>&1
grep median $OUT/ab_wal.txt
step timeout -k 10 300 python -u tools/ab_run.py shards 2 ablibs/libewal_N.so ablibs/libewal_I0.so ablibs/libewal_I2.so ablibs/libewal_I4.so > $OUT/ab_shards.txt 2>&1
grep median $OUT/ab_shards.txt
step timeout -k 10 200 python -u tools/ab_run.py c1 2 ablibs/libewal_N.so ablibs/libewal_I2.so > $OUT/ab_c1.txt 2>&1
grep median $OUT/ab_c1.txt
cat $OUT/steps.txt
