# A/B of ablibs/libewal_A.so vs libewal_B.so on one box (bench wal + shards at 128), 3 alternating rounds
set -e
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_B.so" ${1:-3} "${2:-wal shards}" > gpurun_out/ab.log 2>&1
