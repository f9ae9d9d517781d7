# A/B: M = the regular path's end event recorded behind the last kernel (one device wait per call), vs L; GPU suite on M
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_L.so ablibs/libewal_M.so" 3 "c1 wal" > gpurun_out/ab33.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_M.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu33.txt 2>&1
