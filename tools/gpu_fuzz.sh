#!/bin/bash
# The fuzz suite and a longer run of its tile-spanning large-WAL case
# (tools/fuzz_long.py).  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/fuzz}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -m gpu \
  > "$out/pytest_fuzz.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 1000 ${2:-400} > "$out/fuzz_long.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 5000 ${3:-100} --batch > "$out/fuzz_long_batch.txt" 2>&1
timeout -k 10 600 python3 -u tools/fuzz_long.py 8000 ${4:-100} --split > "$out/fuzz_long_split.txt" 2>&1
echo done
