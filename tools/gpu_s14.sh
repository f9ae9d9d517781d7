#!/bin/bash
# Round-5 session 14: the frame pass's 128-B prefixes (vh[]) -- their parity
# tests first, then the whole GPU suite, then A/B against the build without
# them (auto mode: on from the second call for record-dense WALs).
set -eo pipefail
out=${1:-gpurun_out/s14}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_vh.py -x -v --timeout 300 --timeout-method thread \
  > "$out/pytest_vh.txt" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_cur.so ablibs/libewal_vh.so > "$out/ab_vh_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 2 ablibs/libewal_cur.so ablibs/libewal_vh.so > "$out/ab_vh_wal.txt" 2>&1
echo done
