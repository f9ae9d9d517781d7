#!/bin/bash
# r03 call k: GPU suite (split byte fields, torn shard tails in the batch pass, grouped k_cand),
# A/B of k_cand grouping and k_fc occupancy vs the previous build, the torn5 / restart lines
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -3 $OUT/pytest.txt
grep -q " passed" $OUT/pytest.txt && ! grep -qE "failed|error" $OUT/pytest.txt || exit 1
step bash tools/gpu_ab.sh r03k "wal:3 shards:2 c1:2" ablibs/libewal_N.so ablibs/libewal_C.so ablibs/libewal_F512.so ablibs/libewal_F1024.so
step timeout -k 10 300 python -u bench.py --workload shards --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_shards.json 2> $OUT/bench_shards.err
tail -c 600 $OUT/bench_shards.json
step timeout -k 10 300 python -u bench.py --workload restart --steps 3 > $OUT/bench_restart.json 2> $OUT/bench_restart.err
tail -c 800 $OUT/bench_restart.json
cat $OUT/steps.txt
