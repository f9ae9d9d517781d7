#!/bin/bash
# Round-5 session 18: the driver's N=2 command rehearsed on the one-GPU box
# (both ranks on cuda:0, gloo carrying the same all-reduces and barriers the
# RCCL run does): every sub-config must run with two ranks.
set -eo pipefail
out=${1:-gpurun_out/s18}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --one-device --dist-backend gloo --steps 5 --warmup 1 \
  > "$out/bench_n2.json" 2> "$out/bench_n2.err"
echo done
