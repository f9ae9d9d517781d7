# A/B: D = HEAD; F1 = v[] nontemporal stores; F2 = contiguous tile runs in the single-WAL k_fc too
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_D.so ablibs/libewal_F1.so ablibs/libewal_F2.so" 3 "wal shards" > gpurun_out/ab26.log 2>&1
