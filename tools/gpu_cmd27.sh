# A/B: G = k_stream / k_fc issue their first loads before staging the LDS tables, vs D (HEAD); GPU suite on G
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_D.so ablibs/libewal_G.so" 3 "wal shards" > gpurun_out/ab27.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_G.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu27.txt 2>&1
