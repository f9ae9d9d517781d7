#!/bin/bash
# r03 call p: the within-file split and range-info GPU tests again, then the whole GPU suite; k_commit ILP A/B
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 400 python -u -m pytest tests/test_split_within_file.py tests/test_split_wal.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_split.txt 2>&1
tail -4 $OUT/pytest_split.txt
step timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -3 $OUT/pytest.txt
for r in 1 2; do for L in M1 M2 M4 M8; do
  EWAL_LIB_PATH=ablibs/libewal_$L.so timeout -k 10 120 python3 bench.py --workload commit --steps 50 --no-cpu-baseline > $OUT/commit_$L.$r.json 2>/dev/null
  echo "rc=$?: commit $L $r" >> $OUT/steps.txt
  python3 -c "import json,sys; d=json.loads(open('$OUT/commit_$L.$r.json').read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
cat $OUT/steps.txt
