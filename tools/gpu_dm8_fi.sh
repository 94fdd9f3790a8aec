# dm8 with F/I wave roles in the steady state and one token per wave in the fill and drain
# (make exp NAME=fi DEFS=-DBCFFT_DM8_FI): interleaved A/B against the product, bitwise output
# comparison, then the dm8 parity tests on the experiment library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fi || exit 1
L=$PWD/llama-fft_amd/lib
for r in 1 2; do
  BCFFT_LIB_PATH=$L/libbcfft.so timeout -k 10 200 python -u tools/ab_dm8.py prod$r /tmp/fi_out >> gpurun_out/fi/ab.log 2>&1 || exit 1
  BCFFT_LIB_PATH=$L/libbcfft_exp_fi.so timeout -k 10 200 python -u tools/ab_dm8.py fi$r /tmp/fi_out >> gpurun_out/fi/ab.log 2>&1 || exit 1
done
timeout -k 10 100 python -u tools/ab_dm8.py --compare /tmp/fi_out prod1 fi1 >> gpurun_out/fi/ab.log 2>&1 &&
BCFFT_LIB_PATH=$L/libbcfft_exp_fi.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_0_north_star.py tests/test_gpu_glu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/fi/pytest.log 2>&1
