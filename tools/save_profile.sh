#!/bin/bash
# Archive the last gpu_cycle.sh results under profiles/<round>/<name>_*.
# Usage: tools/save_profile.sh r01 v2
set -e
cd /root/repo
d=profiles/$1; n=$2; mkdir -p $d
grep -v amdgpu.ids gpurun_out/bench.log > $d/${n}_bench.json
cp gpurun_out/prof/stats_kernel_stats.csv $d/${n}_kernel_stats.csv
[ -d gpurun_out/pmc ] && python3 tools/pmc_summary.py gpurun_out/pmc > $d/${n}_pmc.txt || true
[ -f gpurun_out/membw.log ] && cp gpurun_out/membw.log $d/${n}_membw.txt || true
ls $d
