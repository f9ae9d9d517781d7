#!/bin/bash
# The final build's GPU suite, smoke, the default bench line
# and the kernel stats of every workload.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/final}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1
timeout -k 10 600 python3 bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
p="$out/prof"
mkdir -p "$p"
for w in wal c1 shards snap commit rewind; do
  bash tools/prof_kernels.sh "$p/$w" $w --configs none > "$p/$w.summary.txt"
  cp "$(find "$p/$w" -name '*kernel_stats.csv' | head -1)" "$p/${w}_kernel_stats.csv"
done
echo done
