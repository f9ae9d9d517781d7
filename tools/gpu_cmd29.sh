# A/B: I = G + k_uagg's first tile loads in flight during its table staging, vs G; GPU suite on I
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_G.so ablibs/libewal_I.so" 3 "wal shards" > gpurun_out/ab29.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_I.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu29.txt 2>&1
