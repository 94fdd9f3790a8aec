# A/B of a dm8 experiment library (default libbcfft_exp_fi.so: F/I wave roles in the steady state
# and one token per wave in the fill and drain, make exp NAME=fi DEFS=-DBCFFT_DM8_FI) against the
# product: interleaved timing rounds, bitwise output comparison, then the dm8 parity tests on the
# product library. usage: bash tools/gpu_dm8_fi.sh [LIB] [TAG]
set -o pipefail
LIB=${1:-libbcfft_exp_fi.so}; TAG=${2:-fi}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
L=$PWD/llama-fft_amd/lib
for r in 1 2; do
  BCFFT_LIB_PATH=$L/libbcfft.so timeout -k 10 200 python -u tools/ab_dm8.py prod$r /tmp/${TAG}_out >> gpurun_out/$TAG/ab.log 2>&1 || exit 1
  BCFFT_LIB_PATH=$L/$LIB timeout -k 10 200 python -u tools/ab_dm8.py exp$r /tmp/${TAG}_out >> gpurun_out/$TAG/ab.log 2>&1 || exit 1
done
timeout -k 10 100 python -u tools/ab_dm8.py --compare /tmp/${TAG}_out prod1 exp1 >> gpurun_out/$TAG/ab.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_0_north_star.py tests/test_gpu_glu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
