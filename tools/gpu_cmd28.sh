# A/B: H = G + the seam kernel's edge-frame shifts from LDS nibble tables, vs G; GPU suite on H
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_G.so ablibs/libewal_H.so" 3 "wal shards" > gpurun_out/ab28.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_H.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu28.txt 2>&1
