#!/bin/bash
# Round-5 session: the overlapped pipeline's A/B sweep (hooks build, EWAL_OV)
# and the GPU suite on the product build.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s2}
mkdir -p "$out"
export TMPDIR=/tmp
L=ablibs/libewal_hooks.so
timeout -k 10 300 python3 -u tools/env_sweep.py wal 2 $L EWAL_OV=0 EWAL_OV=8,32 EWAL_OV=8,48 EWAL_OV=16,32 \
  EWAL_OV=4,32 EWAL_OV=8,24 > "$out/ov_sweep.txt" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
echo done
