# A/B: P2 = single-WAL ents with nontemporal stores (batched path unchanged), vs P0 (HEAD); GPU suite + smoke on P2
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_P0.so ablibs/libewal_P2.so" 3 "wal shards" > gpurun_out/ab36.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_P2.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu36.txt 2>&1
