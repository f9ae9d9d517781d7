# full GPU suite + smoke on HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu18.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/pytest_gpu18.txt 2>&1
