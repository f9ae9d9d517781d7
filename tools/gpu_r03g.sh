#!/bin/bash
# r03 call g: the GPU suite (residual Message / snapshot encodings), then k_cand A/B on configs[2]
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -5 $OUT/pytest.txt
step timeout -k 10 300 python -u tools/ab_run.py shards 3 ablibs/libewal_N.so ablibs/libewal_K.so > $OUT/ab_shards.txt 2>&1
grep median $OUT/ab_shards.txt
step timeout -k 10 200 python -u tools/ab_run.py wal 2 ablibs/libewal_N.so ablibs/libewal_K.so > $OUT/ab_wal.txt 2>&1
grep median $OUT/ab_wal.txt
cat $OUT/steps.txt
