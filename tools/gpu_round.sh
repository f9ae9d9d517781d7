#!/bin/bash
# One GPU round trip on the box (run through gpurun from the repo root):
#   GPU tests -> the default bench line (every BASELINE config) -> rocprof
#   kernel stats of the headline and of configs[2].
# Usage (here): /usr/local/graft/bin/gpurun --timeout 1100 -- tools/gpu_round.sh TAG [STAGES]
#   STAGES: any of t (tests) b (bench) p (rocprof), default "tbp"
set -o pipefail
TAG=${1:-run}
STAGES=${2:-tbp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ $STAGES == *t* ]]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -2 "$OUT/pytest_gpu.txt"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { cat "$OUT/smoke.txt"; exit 1; }
fi
if [[ $STAGES == *b* ]]; then
  timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -30 "$OUT/bench.err"; exit 1; }
  tail -c 400 "$OUT/bench.json"
fi
if [[ $STAGES == *p* ]]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wal" -o stats -- \
    python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-e2e --configs none > "$OUT/prof_wal.log" 2>&1 \
    || { tail -20 "$OUT/prof_wal.log"; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_shards" -o stats -- \
    python3 bench.py --workload shards --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_shards.log" 2>&1 \
    || { tail -20 "$OUT/prof_shards.log"; exit 1; }
fi
echo "gpu_round $TAG done"
