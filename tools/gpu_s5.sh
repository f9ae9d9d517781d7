#!/bin/bash
# Round-5 session 5: A/B of the unified prefix tail (base vs tail), the
# FETCH_SIZE calibration of per-lane gathers, the GPU suite and the restart
# E2E line (its own process).  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s5}
mkdir -p "$out"
export TMPDIR=/tmp
for m in wal c1 shards; do
  timeout -k 10 400 python3 -u tools/ab_run.py $m 3 ablibs/libewal_base.so ablibs/libewal_tail.so > "$out/ab_tail_$m.txt" 2>&1
done
timeout -k 10 60 ./tools/gather_cal > "$out/gather_cal.txt" 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/gcal" -o pmc -- ./tools/gather_cal \
  > "$out/gather_cal_pmc.log" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 300 python3 bench.py --workload restart --steps 3 --warmup 1 > "$out/restart.json" 2> "$out/restart.err"
echo done
