# v[] stores: one 128-B line per pair (H), nontemporal (I) vs HEAD (A) and no stores (F), one box
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab_crcstream.py ablibs/libewal_A.so ablibs/libewal_F.so ablibs/libewal_H.so ablibs/libewal_I.so > gpurun_out/ab17.log 2>&1
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_H.so ablibs/libewal_I.so" 2 "wal shards" >> gpurun_out/ab17.log 2>&1
