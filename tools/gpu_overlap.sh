#!/bin/bash
# Kernel timelines of the overlapped pipeline (hooks build)
# and the GPU suite on the product build.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s3}
mkdir -p "$out"
export TMPDIR=/tmp
export EWAL_LIB_PATH=$PWD/ablibs/libewal_hooks.so
for v in "0" "8,32" "8,48" "4,64"; do
  tag=${v/,/_}
  EWAL_OV=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/tr_$tag" -o run -- \
    python3 tools/ov_child.py > "$out/tr_$tag.log" 2>&1
  python3 tools/ov_timeline.py "$out/tr_$tag" 1 > "$out/timeline_$tag.txt"
done
EWAL_OV=8,32 EWAL_OV_NOFR=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/tr_nofr" -o run -- \
  python3 tools/ov_child.py > "$out/tr_nofr.log" 2>&1
python3 tools/ov_timeline.py "$out/tr_nofr" 1 > "$out/timeline_nofr.txt"
unset EWAL_LIB_PATH
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
echo done
