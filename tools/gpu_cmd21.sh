# k_fc ablations (timing only): 16 no failure reports, +1 no seed shift, +2 no prefixes, +8 no ents stores
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/fc_ablate.py 16,17,18,19,24,27 > gpurun_out/fc_ablate21.log 2>&1
