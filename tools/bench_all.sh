#!/bin/bash
# Every bench workload once (ON the GPU box, from the repo root), each line to
# gpurun_out/bench_<workload>.json, plus a rocprofv3 kernel-stats pass per
# workload under gpurun_out/prof_<workload>/.  Stops at the first failure.
# Usage: tools/bench_all.sh [workloads...]
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
WS=${*:-"wal c1 shards snap commit msg snapstream"}
for w in $WS; do
  echo "== $w $(date +%T)"
  timeout -k 10 420 python3 -u bench.py --workload $w --cpu-seconds 8 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  tail -c 600 gpurun_out/bench_$w.json
  if [ "$w" != snapstream ] && [ "$w" != restart ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$w -o run -- \
      python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_$w.log 2>&1
  fi
done
echo "== done $(date +%T)"
