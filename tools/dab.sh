export TMPDIR=/tmp
mkdir -p gpurun_out/dab
for ab in 0 256 512 1024 1792; do
  EWAL_STREAM_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dab/a$ab -o s -- python3 tools/decode_ablate.py 4 > gpurun_out/dab/a$ab.log 2>&1 || exit 1
done
