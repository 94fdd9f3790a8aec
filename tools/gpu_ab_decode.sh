# A/B of the K-chunk kernels' decode sizes and the streamed shapes: product library (write-through
# y stores in dmk / dm64k) against a build with every stream policy off (make exp NAME=p0
# DEFS=-DBCFFT_STREAM_POLICY=0). Both through ctypes (BCFFT_LIB_PATH) so the host path is the same.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abd
L=llama-fft_amd/lib
for r in 1 2; do
  for v in libbcfft libbcfft_exp_p0; do
    BCFFT_LIB_PATH=$PWD/$L/$v.so timeout -k 10 200 python -u tools/time_algos.py auto --downsmall > gpurun_out/abd/ds_${v}_$r.log 2>&1 || exit 1
  done
done
for v in libbcfft libbcfft_exp_p0; do
  BCFFT_LIB_PATH=$PWD/$L/$v.so timeout -k 10 200 python -u tools/ab_stream.py > gpurun_out/abd/ab_${v}.log 2>&1 || exit 1
done
