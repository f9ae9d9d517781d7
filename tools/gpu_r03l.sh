#!/bin/bash
# r03 call l: k_stream with v[] only for units holding a flagged piece (timing-only ablation, the
# coarse-v upper bound), and the configs[2] line with torn5 decided in the batch pass
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
AB_NOCHECK=1 step bash tools/gpu_ab.sh r03l "wal:3 shards:2" ablibs/libewal_X0.so ablibs/libewal_X16.so
step timeout -k 10 300 python -u bench.py --workload shards --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_shards.json 2> $OUT/bench_shards.err
tail -c 700 $OUT/bench_shards.json
cat $OUT/steps.txt
