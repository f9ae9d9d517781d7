#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "pytest rc=$?"
tail -3 $OUT/pytest_gpu.txt
AB_NOCHECK=1 timeout -k 10 300 python -u tools/ab_run.py shards 2 ablibs/libewal_A.so ablibs/libewal_N.so ablibs/libewal_X2.so ablibs/libewal_X8.so > $OUT/ab_shards.txt 2>&1; echo "ab shards rc=$?"
grep median $OUT/ab_shards.txt
timeout -k 10 200 python -u tools/ab_run.py wal 2 ablibs/libewal_A.so ablibs/libewal_N.so > $OUT/ab_wal.txt 2>&1; echo "ab wal rc=$?"
grep median $OUT/ab_wal.txt
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
tail -c 300 $OUT/bench.json
