#!/bin/bash
# r03 call n: the driver's default bench line on the current build, rocprof kernel stats of configs[1] and configs[2]
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
step() { "$@"; local rc=$?; echo "rc=$rc: $*" >> $OUT/steps.txt; [ $rc -lt 124 ] || exit $rc; return 0; }
step timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
step timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
tail -c 300 $OUT/bench.json
export TMPDIR=/tmp
step timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_wal -o stats -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-e2e --configs none > $OUT/prof_wal.log 2>&1
step timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shards -o stats -- python3 bench.py --workload shards --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_shards.log 2>&1
cat $OUT/steps.txt
