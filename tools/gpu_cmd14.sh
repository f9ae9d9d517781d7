# A/B: grouped candidate filter (B) vs HEAD (A) on wal + shards; k_stream without CRC (C, timing only) vs A
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_B.so" 3 "wal shards" > gpurun_out/ab14.log 2>&1
AB_NOCHECK=1 timeout -k 10 400 python3 tools/ab_stream.py ablibs/libewal_A.so ablibs/libewal_C.so 2 8 >> gpurun_out/ab14.log 2>&1
