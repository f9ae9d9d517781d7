#!/bin/bash
# Build an A/B variant of libewal.so: tools/build_ab.sh NAME [extra hipcc flags]
# -> ablibs/libewal_NAME.so (timing experiments with tools/ab_run.py)
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1
shift
mkdir -p ablibs
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result -Iinclude \
  -o ablibs/libewal_$NAME.so etcd_amd/csrc/ewal_api.hip etcd_amd/csrc/ewal_host.cpp etcd_amd/csrc/ewal_join.cpp "$@"
