# A/B: K = each candidate unit's 64-B slot line zeroed by 32 lanes before the candidate stores (no partial-line write-back), vs J (HEAD)
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_J.so ablibs/libewal_K.so" 3 "wal shards" > gpurun_out/ab31.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_K.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu31.txt 2>&1
