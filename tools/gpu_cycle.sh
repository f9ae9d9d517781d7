#!/bin/bash
# One GPU round trip: GPU tests, bench, rocprof kernel stats (+ PMC passes with PMC=1).
# Usage: [PMC=1] tools/gpu_cycle.sh [extra bench args]
cd /root/repo
rm -rf gpurun_out/pytest_gpu.log gpurun_out/bench.log gpurun_out/prof gpurun_out/pmc
PMCCMD=true
[ "${PMC:-0}" = 1 ] && PMCCMD="tools/pmc_stream.sh gpurun_out/pmc $*"
timeout 2400 /usr/local/graft/bin/gpurun --timeout 900 -- "mkdir -p gpurun_out && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && timeout -k 10 300 python -u bench.py --cpu-seconds 3 $* > gpurun_out/bench.log 2>&1 && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o stats -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e $* > gpurun_out/prof.log 2>&1 && $PMCCMD ${EXTRA:+&& $EXTRA}" 2>&1 | grep "status="
tail -2 gpurun_out/pytest_gpu.log 2>/dev/null
grep -v amdgpu.ids gpurun_out/bench.log 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'k_stream GB/s',d['roofline']['achieved'],'kernel_ms',d['roofline']['kernel_ms'],'pipe_ms',d['pipeline_device_ms'])" 2>/dev/null || tail -5 gpurun_out/bench.log 2>/dev/null
python3 - <<'PY' 2>/dev/null
import csv
rows=list(csv.DictReader(open('gpurun_out/prof/stats_kernel_stats.csv')))
for r in rows[:14]:
    print(r['Name'][:50].ljust(50), r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Percentage'])
PY
[ -d gpurun_out/pmc ] && python3 tools/pmc_summary.py gpurun_out/pmc k_stream
true
