#!/bin/bash
# r03 call m: GPU suite on the coarse-v build (1-KiB lins for units without a flagged piece), A/B vs the fine-v build
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -3 $OUT/pytest.txt
grep -q " passed" $OUT/pytest.txt && ! grep -qE "failed|error" $OUT/pytest.txt || exit 1
step bash tools/gpu_ab.sh r03m "wal:4 shards:2 c1:2" ablibs/libewal_C.so ablibs/libewal_V.so
cat $OUT/steps.txt
