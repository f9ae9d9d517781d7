#!/bin/bash
# r03 call o: the GPU suite with the within-file split (product ranges on 2 and 3 ranks)
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 400 python -u -m pytest tests/test_split_within_file.py tests/test_split_wal.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_split.txt 2>&1
tail -8 $OUT/pytest_split.txt
step timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -3 $OUT/pytest.txt
cat $OUT/steps.txt
