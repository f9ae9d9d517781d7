#!/bin/bash
# Round 6's validation of the final build, ON the GPU box from the repo root:
# the GPU suite, smoke, the default bench line, the kernel stats of every
# workload and the HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of k_stream
# (configs[1]) and k_frames (configs[1], configs[2], configs[0]).
# Usage: tools/gpu_round6.sh OUT   (then python3 tools/traffic.py OUT/tr_* ... locally)
set -eo pipefail
out=${1:-gpurun_out/r6final}
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
q=(--steps 3 --warmup 1 --no-cpu-baseline --no-e2e)
bash tools/traffic.sh "$out/tr_stream_wal" k_stream "${q[@]}" --configs none
bash tools/traffic.sh "$out/tr_frames_wal" k_frames "${q[@]}" --configs none
bash tools/traffic.sh "$out/tr_frames_shards" k_frames --workload shards --steps 2 --warmup 1 --no-cpu-baseline
bash tools/traffic.sh "$out/tr_frames_c1" k_frames --workload c1 "${q[@]}"
echo done
