#!/bin/bash
# r03 call f: k_cand prefetch A/B, then the default bench line
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 300 python -u tools/ab_run.py shards 2 ablibs/libewal_N.so ablibs/libewal_K.so ablibs/libewal_K2.so > $OUT/ab_shards.txt 2>&1
grep median $OUT/ab_shards.txt
step timeout -k 10 200 python -u tools/ab_run.py wal 2 ablibs/libewal_N.so ablibs/libewal_K2.so > $OUT/ab_wal.txt 2>&1
grep median $OUT/ab_wal.txt
step timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
tail -c 300 $OUT/bench.json
cat $OUT/steps.txt
