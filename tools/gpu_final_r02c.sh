# Round-2 final check on HEAD: GPU suite, smoke, the driver's default bench invocation
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final2_pytest_gpu.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.txt 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/final2_default_bench.json 2> gpurun_out/final2_default_bench.err
