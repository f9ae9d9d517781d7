# A/B: Q1 = batched k_fc walks the shards forward along each wave's run of tiles (one binary search per wave), vs Q0 (HEAD); GPU suite on Q1
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_Q0.so ablibs/libewal_Q1.so" 3 "shards" > gpurun_out/ab37.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_Q1.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu37.txt 2>&1
