#!/bin/bash
# Round-5 session 12: the markers between the passes -- the frame pass timed
# from the stream pass's end event (cur) vs its own start event (evf0) vs no
# markers between the kernels at all (hooks build, EWAL_NO_MID_EVENTS; the
# call's own time only) -- and the GPU suite on the current build.
set -eo pipefail
out=${1:-gpurun_out/s12}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py c1 3 ablibs/libewal_evf0.so ablibs/libewal_cur.so > "$out/ab_evt_c1.txt" 2>&1
timeout -k 10 600 python3 tools/ab_run.py wal 3 ablibs/libewal_evf0.so ablibs/libewal_cur.so > "$out/ab_evt_wal.txt" 2>&1
timeout -k 10 600 python3 tools/env_sweep.py c1 3 ablibs/libewal_hooks.so X=0 EWAL_NO_MID_EVENTS=1 > "$out/sweep_evt_c1.txt" 2>&1
timeout -k 10 600 python3 tools/env_sweep.py wal 2 ablibs/libewal_hooks.so X=0 EWAL_NO_MID_EVENTS=1 > "$out/sweep_evt_wal.txt" 2>&1
echo done
