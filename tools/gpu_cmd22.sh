# k_fc ablations: stores / atomics (timing only)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/fc_ablate.py 16,24,48,80,120,127 > gpurun_out/fc_ablate22.log 2>&1
