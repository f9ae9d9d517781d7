# k_frame timing ablations (EWAL_STREAM_ABLATE bits: 256 no tail bytes,
# 512 no Horner, 1024 no stores / header CRC); results are wrong by design.
export TMPDIR=/tmp
mkdir -p gpurun_out/dab
for ab in 0 256 512 768 1024 1792; do
  EWAL_STREAM_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dab/a$ab -o s -- python3 tools/decode_ablate.py 8 > gpurun_out/dab/a$ab.log 2>&1 || exit 1
done
