# A/B: J = I + k_uapply as persistent 16-wave workgroups (tables staged once per CU), vs I; GPU suite on J
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_I.so ablibs/libewal_J.so" 3 "wal shards" > gpurun_out/ab30.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_J.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu30.txt 2>&1
