# A/B: P1 = ents written with nontemporal stores, vs P0 (HEAD); GPU suite on P1
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_P0.so ablibs/libewal_P1.so" 3 "wal c1 shards" > gpurun_out/ab35.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_P1.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu35.txt 2>&1
