#!/bin/bash
# Round 6's long fuzz on the final build (run ON the GPU box from the repo root):
# the batched tile-spanning case repeated (the rewind hint right and stale), with
# the 128-B prefixes automatic and forced on, and the single / split cases.
set -eo pipefail
out=${1:-gpurun_out/fuzz6}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/fuzz_long.py 20000 ${2:-600} --batch --repeat > "$out/fuzz_long_batch_repeat.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 30000 ${3:-400} --batch --repeat --vh > "$out/fuzz_long_batch_repeat_vh.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 40000 ${4:-1500} > "$out/fuzz_long.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 50000 ${5:-300} --split > "$out/fuzz_long_split.txt" 2>&1
echo done
