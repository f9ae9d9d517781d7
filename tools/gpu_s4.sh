#!/bin/bash
# Round-5 session 4: the overlapped pipeline's parameter sweep (hooks build)
# and the GPU suite on the product build.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s4}
mkdir -p "$out"
export TMPDIR=/tmp
L=ablibs/libewal_hooks.so
timeout -k 10 400 python3 -u tools/env_sweep.py wal 2 $L EWAL_OV=0 EWAL_OV=4,32 EWAL_OV=4,40 EWAL_OV=6,36 \
  EWAL_OV=6,40 EWAL_OV=8,40 EWAL_OV=6,44 > "$out/ov_sweep.txt" 2>&1
EWAL_LIB_PATH=$PWD/$L EWAL_OV=6,40 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/tr_6_40" \
  -o run -- python3 tools/ov_child.py > "$out/tr_6_40.log" 2>&1
python3 tools/ov_timeline.py "$out/tr_6_40" 1 > "$out/timeline_6_40.txt"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
echo done
